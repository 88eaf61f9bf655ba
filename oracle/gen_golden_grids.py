"""Record the geometry of the reference's own saved image grids (build container only; TEST
INFRASTRUCTURE, see oracle/__init__).

    python oracle/gen_golden_grids.py     # writes tests/golden/reference_grids.npz

``/root/reference/images/*.jpg`` (and ``images/patch/``) are torchvision ``save_image`` grids the
reference wrote (``interpolation.py:1379-1394``: 5 inputs / reconstructions of 1024² at padding
2 → 5132 × 1028; the partial-fusion sweep's 6 fused images → 6158 × 1028; single fused images
1024 × 1024). Stored per file: its (width, height) and the mean brightness of every pixel column
and row (the padding stripes are black), so that ``tests/test_host.py`` can check
``records.make_grid``'s layout against the reference's files without reading them.
"""
import glob
import os

import numpy as np
from PIL import Image

HERE = os.path.dirname(os.path.abspath(__file__))
OUT = os.path.join(os.path.dirname(HERE), "tests", "golden", "reference_grids.npz")
REF = "/root/reference/images"


def main():
    out = {}
    for f in sorted(glob.glob(os.path.join(REF, "*.jpg")) + glob.glob(os.path.join(REF, "patch",
                                                                                "*.jpg"))):
        a = np.asarray(Image.open(f).convert("RGB"), dtype=np.float32).mean(axis=2)
        key = os.path.relpath(f, REF).replace(os.sep, "__")
        out[f"{key}/size"] = np.array([a.shape[1], a.shape[0]])
        out[f"{key}/col"] = a.mean(axis=0).astype(np.float32)
        out[f"{key}/row"] = a.mean(axis=1).astype(np.float32)
        print(key, a.shape[1], a.shape[0])
    np.savez_compressed(OUT, **out)
    print("wrote", OUT, os.path.getsize(OUT), "bytes")


if __name__ == "__main__":
    main()
