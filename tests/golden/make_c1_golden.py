"""Generate tests/golden/c1_text_frames.npz: config C1 frames of
the reference's `Text` SVO (tests/golden/text_svo.npz) -- 256x256 primary
rays, Main.unity and overview cameras, HLSL and exact stack modes (one Result
frame per camera: it is the same in both modes) -- traced by
the strict-IEEE C oracle (oracle/svo_oracle.c).

These are regression vectors for the oracle and the GPU path (the reference's
own tests hold no hit buffers for IntersectSVO): they pin today's
oracle output so that a compiler, flag or refactor change that alters any bit
of a hit record or of the Result colour is caught, on CPU and on the GPU.

    python tests/golden/make_c1_golden.py
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)

W = H = 256
CASES = [("main", 0), ("main", 1), ("overview", 0), ("overview", 1)]


def frames():
    from oracle import oracle as orc
    from raytracingtest_amd import SVOData
    from raytracingtest_amd.camera import main_camera, main_light, overview_camera
    z = np.load(os.path.join(HERE, "text_svo.npz"))
    svo = SVOData.from_absolute(z["abs_child_ptr"], z["valid_mask"], z["nonleaf_mask"], z["normal_code"])
    osvo = orc.OracleSVO(svo.childDescriptors, svo.attachments)
    out = {}
    for cam_name, mode in CASES:
        cam = main_camera() if cam_name == "main" else overview_camera()
        c2w, inv_proj = cam.uniforms(W, H)
        ocam = orc.make_camera(c2w, inv_proj, (0.5, 0.5), main_light())
        hits, rgba, _ = orc.render(osvo, ocam, W, H, mode)
        key = f"{cam_name}_{'hlsl' if mode == 0 else 'exact'}"
        out[key + "_hits"] = np.frombuffer(hits.tobytes(), np.uint8).reshape(H, W, 24)
        rgba = rgba.reshape(H, W, 4).astype(np.float32)
        if cam_name + "_rgba" in out:   # Result does not depend on the stack mode here: stored once
            assert np.array_equal(out[cam_name + "_rgba"], rgba)
        out[cam_name + "_rgba"] = rgba
    return out


if __name__ == "__main__":
    np.savez_compressed(os.path.join(HERE, "c1_text_frames.npz"), **frames())
