"""profile_logP on the device (k_logp behind gqmap_log_p) against the literal
C restatement (oracle/gqmap_oracle.c orc_log_p), full frames:

  * C4 (Urban3 480x640, super engine L=3 K=11): the node term is node_lp, the
    4x4 full-resolution block sum of node_pot per node
    (gqmap_gpuSuper_mix_entropy.m:152-169);
  * C2 (RubberWhale 388x584, mixture L=1 K=9): node_pot per pixel
    (gqmap_gpu_mixture.m:148-154).

The MAP is the device's own get_map of the reference init and of a
converging state (displacements crossing the border clamps in the first).
Tolerance 1e-10 relative: the device sums per-block partials in a different
order than MATLAB's column sums, and the bicubic is the kernel's fma form.
"""
import numpy as np
import pytest

from tests import _fullsize as F

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("init", ["ref", "tight"])
@pytest.mark.parametrize("cfg", ["c4", "c2"])
def test_logp_fullsize_vs_literal(cfg, init):
    from gqmap_opticalflow_amd import Engine
    from oracle import oracle
    I1, I2, _, _, o, st = F.case(cfg, init)
    with Engine(o, I1, I2, o["engine"], "fp64") as eng:
        eng.set_state(st)
        mp = eng.map()
        lp = eng.log_p(mp)
    ref = oracle.log_p(o, I1, I2, mp)
    assert np.isfinite(lp) and lp < 0
    assert lp == pytest.approx(ref, rel=1e-10), (lp, ref)
