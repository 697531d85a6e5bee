"""Per-level diagnostics of the C3 pyramid (device)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402

from gqmap_opticalflow_amd import (C3_SCALES, Pyramid, aepe, ctf_options, flow_to_color, flowio,  # noqa: E402
                                   imresize)

its = int(sys.argv[1]) if len(sys.argv) > 1 else 500
I1, I2, gt = flowio.load_pair("Grove3")
_, flo, (minu, maxu, minv, maxv), unk = flow_to_color(gt)
print("GT range", minu, maxu, minv, maxv)
opts = ctf_options(its=its, minu=minu, maxu=maxu, minv=minv, maxv=maxv)
with Pyramid(opts, C3_SCALES) as p:
    p.set_images(I1, I2)
    flow, done, ms = p.run(seed=0)
    for l, s in enumerate(C3_SCALES):
        g = p.level(l)
        gts = imresize(flo, s) * s
        e = np.sqrt(((g["warp"] - gts) ** 2).sum(2))
        print(f"level {l} s={s}: shape {g['I2'].shape} AEPE(warp) {e[1:-1,1:-1].mean():.3f} "
              f"median {np.median(e):.3f} p99 {np.percentile(e, 99):.2f} "
              f"|flow| max {np.abs(g['flow']).max():.2f} mean {np.abs(g['flow']).mean():.3f} "
              f"warp range u [{g['warp'][:,:,0].min():.2f},{g['warp'][:,:,0].max():.2f}] "
              f"v [{g['warp'][:,:,1].min():.2f},{g['warp'][:,:,1].max():.2f}]", flush=True)
    print("final AEPE", aepe(flo, flow, unk))
