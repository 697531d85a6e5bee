"""Copy the reference's preprocessed (structure-texture) input frames
(middlebury/preprocessed/<name>.mat: img1, img2, fp64 388x584; read by
optical_flowSuper.m:13 when preprocessed=true) into data/middlebury/preprocessed/
as .npz.  scipy.io.loadmat parses the MAT v5 data only.  The generator of
these frames is not in the reference, so the path is pinned on the data alone.
usage: python scripts/make_preprocessed_fixture.py [names...]"""
import os
import sys

import numpy as np
import scipy.io as sio

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = "/root/reference/middlebury/preprocessed"
names = sys.argv[1:] or ["RubberWhale"]
for n in names:
    d = sio.loadmat(os.path.join(SRC, n + ".mat"))
    out = os.path.join(ROOT, "data", "middlebury", "preprocessed", n + ".npz")
    np.savez_compressed(out, img1=np.asarray(d["img1"], np.float64), img2=np.asarray(d["img2"], np.float64))
    print(out, d["img1"].shape, float(d["img1"].min()), float(d["img1"].max()))
