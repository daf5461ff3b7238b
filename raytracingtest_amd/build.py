"""Build the native libraries in-tree (they travel to the GPU box with the repo).

  libsvo_rt.so    : C-ABI + gfx950 HIP kernels (include/svo_rt.h)
  libsvo_build.so : native SVO builder (include/svo_build.h)

hipcc cross-compiles gfx950 without a GPU.  Flags: -ffp-contract=off and no
fast-math so f32 arithmetic rounds exactly like the strict-IEEE oracle.
"""
import os
import shutil
import subprocess
import sys

PKG = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(PKG)
CSRC = os.path.join(PKG, "csrc")
INCLUDE = os.path.join(ROOT, "include")
ARCH = os.environ.get("SVO_OFFLOAD_ARCH", "gfx950")

HIPCC = shutil.which("hipcc") or "/opt/rocm/bin/hipcc"
# -fno-slp-vectorize (device): packed f32 ops (v_pk_mul/add_f32) and the register
# pair copies they need made the traversal loop ~3 % slower (tools/ab_lib.sh).
COMMON = ["-O3", "-std=c++17", "-fPIC", "-shared", "-ffp-contract=off", "-fno-fast-math",
          "-Xarch_device", "-fno-slp-vectorize",
          "-Wno-unused-value", "-Wno-unused-result", "-I" + INCLUDE, "-I" + CSRC]

TARGETS = {
    "libsvo_rt.so": ["svo_rt.hip", "svo_kernel.hip"],
    "libsvo_build.so": ["svo_build.hip"],
}


def _stale(out, srcs):
    if not os.path.exists(out):
        return True
    t = os.path.getmtime(out)
    deps = [os.path.join(CSRC, s) for s in srcs]
    deps += [os.path.join(CSRC, f) for f in os.listdir(CSRC) if f.endswith(".h")]
    deps += [os.path.join(INCLUDE, f) for f in os.listdir(INCLUDE)]
    return any(os.path.getmtime(d) > t for d in deps if os.path.exists(d))


def source_digest(name="libsvo_rt.so"):
    """sha1 over what decides the render kernel's memory traffic -- the library's
    sources (kernels and the launch configuration), the kernel headers and the
    compile flags: the key under which profiling evidence
    (profiles/pmc_summary.json) is valid.  The public C header (include/) is
    left out: its declarations and comments do not change the kernel."""
    import hashlib
    # flags without the include paths: the digest must not depend on where the tree lies
    # (the GPU box runs it from a scratch copy)
    flags = [f for f in COMMON if not f.startswith("-I")]
    h = hashlib.sha1(" ".join(flags + [ARCH]).encode())
    files = [os.path.join(CSRC, s) for s in TARGETS[name]]
    files += sorted(os.path.join(CSRC, f) for f in os.listdir(CSRC) if f.endswith(".h"))
    for f in files:
        with open(f, "rb") as fh:
            h.update(os.path.basename(f).encode())
            h.update(fh.read())
    return h.hexdigest()[:16]


def build(force=False, verbose=False):
    built = []
    for name, srcs in TARGETS.items():
        if not all(os.path.exists(os.path.join(CSRC, s)) for s in srcs):
            continue
        out = os.path.join(PKG, name)
        if not force and not _stale(out, srcs):
            continue
        cmd = [HIPCC, "--offload-arch=" + ARCH] + COMMON + ["-o", out] + [os.path.join(CSRC, s) for s in srcs]
        if verbose:
            print(" ".join(cmd), file=sys.stderr)
        subprocess.run(cmd, check=True)
        built.append(out)
    return built


if __name__ == "__main__":
    build(force="--force" in sys.argv, verbose=True)
