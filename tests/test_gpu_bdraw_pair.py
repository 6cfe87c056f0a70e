"""gs_bdraw_tiled with two chains per wave (k_bdraw_pair, GS_OPT_SWEEP_SCHED = 3) against the one-chain
kernel (GS_OPT_SWEEP_SCHED = 2): bit-identical b, info and failure counts, for Philox and injected
normals, a mixed gate (shut chains keep b and get nothing written), phiinv per chain (curn) and per
system (curn_red, grid-conditional red), and the 45-pulsar array whose two nM = 17 pulsars take the
row-major fixed block (drawn one chain at a time inside the pair kernel; at 128 chains the items outnumber
one round of workgroups, so the cost-weighted persistent ranges run).  Needs an MI355X."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")


def _engine(kind, n_psr, C):
    from pulsar_timing_gibbsspec_amd import PTABlockGibbs, synthetic
    pta = synthetic.array_pta(kind=kind, n_psr=n_psr, seed=5)
    # curn_red with the grid-conditional red block: the default 'mh' attaches the lnL output, whose
    # draws stay on the one-chain kernel
    gb = PTABlockGibbs(pta, nchains=C, seed=13, redsample="conditional" if kind == "curn_red" else "mh")
    x0 = np.concatenate([np.atleast_1d(p.sample()).ravel() for p in gb.params])
    eng = gb._new_engine(x0)
    for _ in range(3):
        eng.sweep()
    return eng


def _draw(eng, sched, z, mask):
    from pulsar_timing_gibbsspec_amd import _lib
    b0 = eng.b.clone()
    eng.info.zero_()
    eng.fail_count.zero_()
    prev = eng.ctx.get_option(_lib.OPT_SWEEP_SCHED)
    eng.ctx.set_option(_lib.OPT_SWEEP_SCHED, sched)
    try:
        eng._bdraw(z, _lib.EV_B, mask)
        shape = eng.ctx.get_option(_lib.OPT_LAST_SWEEP_SHAPE)
    finally:
        eng.ctx.set_option(_lib.OPT_SWEEP_SCHED, prev)
    out = (eng.b.clone(), eng.info.clone(), eng.fail_count.clone(), shape)
    eng.b.copy_(b0)
    return out


@pytest.mark.parametrize("kind,n_psr,C", [("curn", 6, 64), ("curn_red", 6, 38), ("curn", 45, 32), ("curn", 45, 128)])
@pytest.mark.parametrize("inject", [False, True])
def test_bdraw_pair_equals_one_chain(kind, n_psr, C, inject):
    eng = _engine(kind, n_psr, C)
    m = eng.model
    z = None
    if inject:
        z = torch.as_tensor(np.random.default_rng(1).standard_normal((m.P * C, m.ldb)), device="cuda")
    gate = torch.tensor([(c % 5) != 2 for c in range(C)], dtype=torch.int32, device="cuda")
    b0 = eng.b.clone()
    b2, i2, f2, s2 = _draw(eng, 2, z, gate)
    b3, i3, f3, s3 = _draw(eng, 3, z, gate)
    assert (s2, s3) == (2, 3)
    assert torch.equal(b2, b3) and torch.equal(i2, i3) and torch.equal(f2, f3)
    shut = ~gate.bool().repeat(m.P)
    assert torch.equal(b3[shut], b0[shut])                 # shut gates keep their b
    assert not torch.equal(b3[~shut], b0[~shut])
    assert not i3.any() and not f3.any()
    if n_psr == 45:
        assert int(m.NMX) > 16 and int((m.nm_dev > 16).sum()) > 0   # row-major pulsars in the batch


def test_bdraw_pair_failure_keeps_b():
    """A non-PD system in the pair kernel: that chain keeps its b and its info is set, and its pair
    partner draws normally -- as in the one-chain kernel (info, b and any attached failure counts equal)."""
    eng = _engine("curn_red", 3, 8)
    m, C = eng.model, eng.C
    eng.phiinv_F.view(m.P, C, -1)[1, 5, 3] = -1e30        # pulsar 1, chain 5 (partner of chain 4)
    b2, i2, f2, _ = _draw(eng, 2, None, None)
    b3, i3, f3, _ = _draw(eng, 3, None, None)
    assert torch.equal(b2, b3) and torch.equal(i2, i3) and torch.equal(f2, f3)
    sys = 1 * C + 5
    assert int(i3[sys]) > 0
    assert torch.equal(b3[sys], eng.b[sys])
    assert int(i3[sys - 1]) == 0 and not torch.equal(b3[sys - 1], eng.b[sys - 1])
    assert int((i3 != 0).sum()) == 1
