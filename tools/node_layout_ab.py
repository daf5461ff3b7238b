"""Does node DENSITY move the lean loop?  A diagnostic before any node-layout change
("a layout or trip-count change").  Two variant libraries are built from
patched copies of csrc/ (string edits asserted to apply exactly once; nothing in the product
sources changes):

  pad16 : the V2 node pool copied to a 16-byte stride (node i at byte 16 i) -- half the nodes
          per cache line, same loads, same instructions but one shift;
  split : the pool split into a 2-byte mask array and a 4-byte first-child array (6 B per
          node, four times the masks per line) -- two loads per trip instead of one.

Only the lean loop's unpredicated fetch (C1-C3 pools, !GUARD) reads the copy, so every run
forces SVO_LAT=0.  Each variant runs in its own process through SVO_RT_LIB, interleaved
with the product library, on the C3 frame at two poses and the lone heaviest tile row;
its hit records must equal the product library's.

  python tools/node_layout_ab.py build             # here: libraries into build_ab/
  python tools/node_layout_ab.py run [--rounds 2]  # GPU box
  python tools/node_layout_ab.py one <lib>         # one process (what `run` starts)
"""
import hashlib
import os
import shutil
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
OUT = os.path.join(ROOT, "build_ab")

LEAN_FETCH = ": *(const uint2 *)((const char *)p.nodes + (uint32_t)(r.parent << 3));"
VARIANT_FETCH = {
    "pad16": ": *(const uint2 *)((const char *)p.nodes + (uint32_t)(r.parent << 4));",
    "split": (": make_uint2((uint32_t)*(const uint16_t *)((const char *)p.nodes + (uint32_t)(r.parent << 1)),"
              " *(const uint32_t *)((const char *)p.nodes + ((2u * p.n_nodes + 255u) & ~255u)"
              " + (uint32_t)(r.parent << 2)));"),
}
RT_ANCHOR = "    p.nodes = ctx->d_nodes;\n"
RT_KERNEL_ANCHOR = "// Make stream s wait for the work the previous scratch user enqueued on another stream.\n"
RT_KERNEL = r'''
__global__ void diag_layout_kernel(const uint2 *__restrict__ src, char *__restrict__ dst, uint32_t n, int layout) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint2 v = src[i];
    if (layout == 1) {
        reinterpret_cast<uint4 *>(dst)[i] = make_uint4(v.x, v.y, 0u, 0u);
    } else {
        reinterpret_cast<uint16_t *>(dst)[i] = (uint16_t)v.x;
        reinterpret_cast<uint32_t *>(dst + ((2u * n + 255u) & ~255u))[i] = v.y;
    }
}
const uint2 *diag_nodes(svo_ctx *ctx, uint32_t n) {
    static char *buf = nullptr;
    static const void *src = nullptr;
    static uint32_t built_n = 0;
    if (buf && src == ctx->d_nodes && built_n == n) return reinterpret_cast<const uint2 *>(buf);
    hipDeviceSynchronize();
    if (buf) hipFree(buf);
    const size_t bytes = LAYOUT == 1 ? 16ull * n : ((2ull * n + 255) & ~255ull) + 4ull * n;
    if (hipMalloc(&buf, bytes) != hipSuccess) return nullptr;
    hipLaunchKernelGGL(diag_layout_kernel, dim3((n + 255) / 256), dim3(256), 0, 0, ctx->d_nodes, buf, n, LAYOUT);
    hipDeviceSynchronize();
    src = ctx->d_nodes;
    built_n = n;
    return reinterpret_cast<const uint2 *>(buf);
}

'''


def patch(text, old, new):
    assert text.count(old) == 1, f"patch anchor found {text.count(old)} times: {old[:60]!r}"
    return text.replace(old, new)


def build():
    from raytracingtest_amd import build as b
    os.makedirs(OUT, exist_ok=True)
    for layout, name in ((1, "pad16"), (2, "split")):
        src = os.path.join(OUT, "csrc_" + name)
        if os.path.exists(src):
            shutil.rmtree(src)
        shutil.copytree(b.CSRC, src)
        kp = os.path.join(src, "svo_kernel.hip")
        with open(kp) as f:
            k = f.read()
        k = patch(k, LEAN_FETCH, VARIANT_FETCH[name])
        with open(kp, "w") as f:
            f.write(k)
        rp = os.path.join(src, "svo_rt.hip")
        with open(rp) as f:
            r = f.read()
        r = patch(r, RT_KERNEL_ANCHOR, f"#define LAYOUT {layout}\n" + RT_KERNEL + RT_KERNEL_ANCHOR)
        r = patch(r, RT_ANCHOR, RT_ANCHOR +
                  "    if (!ctx->depth_exact || ctx->n_nodes >= ((size_t)1 << 24)) return fail(SVO_ERR_ARG, \"diag layout: C1-C3 pools only\");\n"
                  "    p.nodes = diag_nodes(ctx, (uint32_t)ctx->n_nodes);\n")
        with open(rp, "w") as f:
            f.write(r)
        flags = [c for c in b.COMMON if not c.startswith("-I")] + ["-I" + b.INCLUDE, "-I" + src]
        lib = os.path.join(OUT, f"libsvo_rt_{name}.so")
        cmd = [b.HIPCC, "--offload-arch=" + b.ARCH] + flags + ["-o", lib,
                                                              os.path.join(src, "svo_rt.hip"), os.path.join(src, "svo_kernel.hip")]
        subprocess.run(cmd, check=True)
        shutil.rmtree(src)
        print("built", lib)


def one(lib):
    os.environ["SVO_LAT"] = "0"
    if lib != "product":
        os.environ["SVO_RT_LIB"] = os.path.join(OUT, f"libsvo_rt_{lib}.so")
    import torch
    from bench import CONFIGS
    from raytracingtest_amd import RaytracingMaster
    from raytracingtest_amd.camera import CAMERAS
    from raytracingtest_amd.native_builder import build_sampler_svo
    cfg = CONFIGS["C3"]
    W, H = cfg["width"], cfg["height"]
    svo = build_sampler_svo(cfg["sampler"], cfg["max_level"])
    rm = RaytracingMaster(capacity_nodes=len(svo))
    rm.SetSVOBuffer(svo)
    s = torch.cuda.Stream()
    out = [lib]
    for cam, band, warm, reps in (("flyover", None, 300, 500), ("main", None, 200, 300),
                                  ("flyover", (8, 80, (H + 7) // 8), 20, 50)):
        rm.UpdateShaderParameters(CAMERAS[cam](), W, H)
        rows = 8 if band else H
        h = torch.empty(rows * W * 24, dtype=torch.uint8, device="cuda")
        rgba = None if band else torch.empty(rows * W * 4, dtype=torch.float32, device="cuda")
        torch.cuda.synchronize()

        def go():
            rm.render_device(W, H, hits_ptr=h.data_ptr(), rgba_ptr=None if rgba is None else rgba.data_ptr(),
                             band=band, stack_mode=0, stream=s.cuda_stream)
        for _ in range(warm):
            go()
        torch.cuda.synchronize()
        rm.set_kernel_timing(True)
        rm.kernel_time()
        for _ in range(reps):
            go()
        ms, n = rm.kernel_time()
        rm.set_kernel_timing(False)
        torch.cuda.synchronize()
        digest = hashlib.sha1(h.cpu().numpy().tobytes()).hexdigest()[:12]
        out.append(f"{cam}{'/row80' if band else ''} {ms * 1e3:.2f}us hits:{digest}")
    print(" | ".join(out), flush=True)
    rm.close()


def run(rounds):
    for r in range(rounds):
        for lib in ("product", "pad16", "split"):
            subprocess.run([sys.executable, os.path.abspath(__file__), "one", lib], check=True, timeout=300)


if __name__ == "__main__":
    if sys.argv[1] == "build":
        build()
    elif sys.argv[1] == "one":
        one(sys.argv[2])
    else:
        run(int(sys.argv[sys.argv.index("--rounds") + 1]) if "--rounds" in sys.argv else 2)
