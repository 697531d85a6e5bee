"""Full-frame HIP parity on the BASELINE configs' own frames (see
tests/_fullsize.py): C2 RubberWhale 388x584 mixture, C3's finest Grove3
480x640 ctf level, C4 Urban3 480x640 super L=3 K=11.

  * one iteration, fp64: within 1e-10 of the literal restatement of the
    MATLAB (oracle/gqmap_oracle.c) and bit-identical to the CPU model of
    the kernel arithmetic (oracle/gqmap_emul.cpp), from the reference init
    and from a converging state where the fast paths carry >90% of the work;
  * fp32: bit-identical to the fp32 CPU model;
  * the C4 workload with its schedule compressed (alpha update after
    iteration 20, temperature decay every 20) over 60 iterations, softmax and
    projsplx, bit-identical to the CPU model.
"""
import os

import numpy as np
import pytest

from tests import _fullsize as F
from tests import _golden as G

pytestmark = pytest.mark.gpu
NT = min(16, os.cpu_count() or 1)


def _gh(K):
    from gqmap_opticalflow_amd import gauss_hermite
    return gauss_hermite(K)


def _gpu(o, I1, I2, st, its, precision="fp64"):
    from gqmap_opticalflow_amd import Engine
    with Engine(o, I1, I2, o["engine"], precision) as eng:
        eng.set_state(st)
        done, tr = eng.run(its)
        return done, tr, eng.get_state(), eng.info().split


def _emu(o, I1, I2, st, its, split, precision="fp64"):
    from oracle import oracle
    ost = F.oracle_state(st)
    X, W = _gh(o["K"])
    done, tr, T = oracle.emu_run(o, I1, I2, ost, st.it, its, X, W, T=st.T, nthreads=NT,
                                 fp32=precision == "fp32", split=split)
    return done, tr, T, ost


def _bit_exact(g, tr, done, e):
    e_done, e_tr, _, ost = e
    assert done == e_done
    np.testing.assert_array_equal(tr, e_tr)
    for k, a in zip(G.STATE_KEYS, ost.arrays()):
        np.testing.assert_array_equal(getattr(g, k), a, err_msg=k)


@pytest.mark.parametrize("init", ["ref", "tight"])
@pytest.mark.parametrize("cfg", ["c2", "c3", "c4"])
def test_fullsize_one_iteration_vs_literal_and_emulator(cfg, init):
    from oracle import oracle
    I1, I2, _, _, o, st = F.case(cfg, init)
    done, tr, g, split = _gpu(o, I1, I2, st, 1)
    lit = F.oracle_state(st)
    n, tr_lit, _ = oracle.run(o, I1, I2, lit, 1, 1, nthreads=NT)
    assert done == n == 1
    np.testing.assert_allclose(tr, tr_lit, rtol=1e-10)
    for k, a in zip(G.STATE_KEYS, lit.arrays()):
        np.testing.assert_allclose(getattr(g, k), a, rtol=1e-10, atol=1e-10, err_msg=k)
    _bit_exact(g, tr, done, _emu(o, I1, I2, st, 1, split))


@pytest.mark.parametrize("cfg", ["c2", "c4"])
def test_fullsize_fp32_bit_exact_vs_emulator(cfg):
    I1, I2, _, _, o, st = F.case(cfg, "tight")
    done, tr, g, split = _gpu(o, I1, I2, st, 3, "fp32")
    _bit_exact(g, tr, done, _emu(o, I1, I2, st, 3, split, "fp32"))


@pytest.mark.parametrize("mode", [0, 1])
def test_c4_workload_compressed_schedule_bit_exact(mode):
    """BASELINE C4 (Urban3 480x640 super, L=3, K=11, T=0.2, drate=0.75,
    lambdas=16) with the reference schedule compressed 25x: alpha update
    after iteration 20 (softmax: updateAlpha; projsplx: the mode's reference
    step scale 1E-6) and T decay every 20 iterations, 60 iterations."""
    I1, I2, _, _, o, st = F.case("c4", "ref", alpha_mode=mode, alpha_start=20, t_decay_every=20)
    its = 60
    done, tr, g, split = _gpu(o, I1, I2, st, its)
    e = _emu(o, I1, I2, st, its, split)
    _bit_exact(g, tr, done, e)
    assert done == its
    assert g.T == e[2] == pytest.approx(0.2 * 0.75 ** 3)
    assert not np.array_equal(g.alpha, st.alpha)  # the alpha update ran
    assert g.alpha.sum() == pytest.approx(1.0)


@pytest.mark.parametrize("cfg", ["c2_dimetrodon", "c2_hydrangea"])
def test_fullsize_other_pairs_20_iterations_bit_exact(cfg):
    # the frames the multi-GPU frame-parallel ranks solve (bench.PAIRS):
    # 20 fp64 iterations bit-identical to the CPU model
    I1, I2, _, _, o, st = F.case(cfg, "ref")
    done, tr, g, split = _gpu(o, I1, I2, st, 20)
    assert split == 1
    _bit_exact(g, tr, done, _emu(o, I1, I2, st, 20, split))
