"""Bring-up check on the GPU box: HIP path vs oracle on small configs (both kernel variants)."""
import sys, os, time
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests"))
from helpers import SceneCase, mismatch_report, _lib
import numpy as np
ok = True
for name, size, S, B in [("cube", (256, 256), 1, 1), ("box", (128, 128), 4, 4), ("island", (160, 90), 4, 8),
                         ("cave", (96, 54), 2, 8), ("spheres", (80, 60), 2, 8), ("box", (37, 23), 3, 5)]:
    case = SceneCase(name, size, S, B)
    t = time.time(); ref, _, seg, tt = case.oracle(); tcpu = time.time() - t
    for variant in (1, 0):
        img, gseg, gtt = case.gpu(variant=variant)
        same = np.array_equal(img, ref)
        ok &= same and gseg == seg and gtt == tt
        print(f"{name:8s} {size} S={S} B={B} variant={variant}: {mismatch_report(img, ref)}; "
              f"segments gpu={gseg} cpu={seg}; tests gpu={gtt} cpu={tt}; oracle {tcpu:.2f}s", flush=True)
print("ALL OK" if ok else "MISMATCH")
sys.exit(0 if ok else 1)
