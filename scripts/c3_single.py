import os, sys
sys.path.insert(0, '.')
import numpy as np
from gqmap_opticalflow_amd import gqmap_ctf, gqmap_gpu_mixture, flow_to_color, flowio, aepe
I1, I2, gt = flowio.load_pair("Grove3")
_, flo, (minu, maxu, minv, maxv), unk = flow_to_color(gt)
for its in (200, 1000):
    mu, sg, rou, A, E = gqmap_ctf(dict(K=11, its=its, epsn=1e-6, lambdas=5, lambdad=1), I1, I2, flo)
    print("ctf single level its", its, "AEPE(GT unk->0)", aepe(flo, mu, unk), "ref-style", A[~np.isnan(A)][-1], flush=True)
o = dict(its=500, K=9, L=1, temperature=0, drate=0.5, epsn=1e-6, lambdas=5, lambdad=1, minu=minu, maxu=maxu, minv=minv, maxv=maxv, trueFlow=flo, unknownIdx=unk)
mu, sigma, alpha, AEPE, Energy, logP = gqmap_gpu_mixture(o, I1, I2)
print("mixture 500 its AEPE", AEPE[~np.isnan(AEPE)])
