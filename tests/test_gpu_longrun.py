"""Long-run parity of the HIP path against the LITERAL restatement
(oracle/gqmap_oracle.c: the reference's own operation order, libm sqrt),
BASELINE config C2 (RubberWhale 388x584, gqmap_gpu_mixture, L=1, K=9).

The GPU is bit-identical to the CPU model of its own arithmetic for any
number of iterations (test_gpu_parity.py).  Against the literal
restatement the per-step agreement is ~1e-12 (test_fullsize.py), and the
solver's chaotic transient amplifies that: a 1e-13 perturbation of the
initial state already moves iteration 10's Energy by ~2e-6 relative, and
the end-state AEPE after 300 iterations of the literal restatement itself
spreads over 2.504 .. 2.517 (sigma ~0.006) under perturbations of 1e-13 and
2e-13 (profiles/r03_longrun_spread.txt).  Long-run parity with the reference
is therefore tolerance-based, with the tolerances written here:
  * iteration 1 (before any amplification): trace within 1e-10 relative;
  * after 300 iterations: |AEPE(GPU) - AEPE(literal)| <= 0.02 (about 3 sigma
    of the literal restatement's own spread).  Both sides are deterministic,
    so the test is too: it does not flake, it only moves with the spec.
The stop rule (ptdmu < tor, gqmap_gpu_mixture.m:75) is not pinned by a long
run: at the reference settings ptdmu stays O(10) for thousands of
iterations, so no run here stops; the rule itself is tested where it fires
(test_gpu_parity.py::test_stop_rule_ptdmu_below_tor, ::test_stop_inside_a_graph_chunk).
"""
import numpy as np
import pytest

from tests import _fullsize as F

pytestmark = pytest.mark.gpu


def test_c2_300_iterations_aepe_vs_literal_restatement():
    from gqmap_opticalflow_amd import Engine, aepe
    from oracle import oracle
    I1, I2, flo, unk, o, st = F.case("c2")
    its = 300
    with Engine(o, I1, I2) as eng:
        eng.set_state(st)
        done, tr = eng.run(its)
        a_gpu = aepe(flo, eng.map(), unk)
    ost = F.oracle_state(st)
    odone, otr, _ = oracle.run(o, I1, I2, ost, 1, its, nthreads=16)
    a_lit = aepe(flo, np.stack([ost.muu[:, :, 0], ost.muv[:, :, 0]], axis=2), unk)
    print(f"AEPE after {its} its: gpu={a_gpu:.6f} literal={a_lit:.6f}")
    assert done == odone == its
    np.testing.assert_allclose(tr[0], otr[0], rtol=1e-10)
    assert abs(a_gpu - a_lit) <= 0.02
