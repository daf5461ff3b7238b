"""Debug aid for the refill experiment: mismatching pixels vs the default kernel."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    from raytracingtest_amd import RaytracingMaster, HIT_DTYPE
    from raytracingtest_amd.builder import build_menger
    from raytracingtest_amd.camera import overview_camera
    svo = build_menger(8)
    w, h = 333, 201
    res = {}
    for env in ("", "2,16", "1,64", "1,1", "2,64"):
        if env:
            os.environ["SVO_REFILL"] = env
        else:
            os.environ.pop("SVO_REFILL", None)
        m = RaytracingMaster(device=0, capacity_nodes=len(svo))
        m.SetSVOBuffer(svo)
        m.UpdateShaderParameters(overview_camera(), w, h)
        rgba, hits = m.Render(w, h)
        m.close()
        res[env] = hits.reshape(h, w)
    ref = res[""]
    for env, hh in res.items():
        if not env:
            continue
        bad = np.argwhere(hh.view(np.uint8).reshape(h, w, 24).any(2) & (hh.view(np.uint8).reshape(h, w, 24) != ref.view(np.uint8).reshape(h, w, 24)).any(2))
        print(env, "mismatches", len(bad), "of", w * h, "hits ref", int((ref["flags"] & 1).sum()), "got", int((hh["flags"] & 1).sum()))
        for y, x in bad[:6]:
            print("   ", y, x, "ref", ref[y, x], "got", hh[y, x])


if __name__ == "__main__":
    main()
