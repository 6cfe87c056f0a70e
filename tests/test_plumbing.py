"""Host-side plumbing on CPU (no GPU: the device context is created on first use).

Parameter names / order, the vector <-> dict map, prior bounds parsed from str(param),
the gw / ECORR column walk and the pulsar sharding, checked against the reference's own
outputs stored in the golden fixtures (param_names, b_param_names, gwid, rho bounds).
"""
import numpy as np
import pytest

from tests.conftest import golden


def test_pulsar_block_gibbs_plumbing_matches_reference(single):
    from pulsar_timing_gibbsspec_amd import PulsarBlockGibbs, synthetic
    gb = PulsarBlockGibbs(synthetic.single_pulsar_pta("J1713+0747", seed=0), seed=1)
    assert gb.param_names == list(single["param_names"])
    assert gb.b_param_names == list(single["b_param_names"])
    assert np.array_equal(gb.gwid, single["gwid"])
    assert (gb.rhomin, gb.rhomax) == (float(single["rhomin"]), float(single["rhomax"]))
    d = gb.map_params(single["x0"])
    assert list(d) == ["gw_log10_rho"] and np.array_equal(d["gw_log10_rho"], single["x0"])
    assert np.array_equal(gb.get_gwrho_param_indices(), np.arange(30))
    assert gb.get_red_param_indices().size == 0 and gb.get_efacequad_indices().size == 0


def test_white_and_ecorr_plumbing_matches_reference():
    from pulsar_timing_gibbsspec_amd import PulsarBlockGibbs, synthetic
    g = golden("ecorr_white_j1713.npz")
    gb = PulsarBlockGibbs(synthetic.ecorr_pulsar_pta("J1713+0747", seed=0, white_vary=True), seed=1)
    assert gb.param_names == list(g["param_names"])
    assert np.array_equal(gb.ecid, g["ecid"]) and np.array_equal(gb.gwid, g["gwid"])
    assert np.array_equal(gb.get_ecorr_indices(), g["eind"])
    assert np.array_equal(gb.get_efacequad_indices(), g["wind"])


@pytest.mark.parametrize("kind", ["curn", "curn_red"])
def test_pta_block_gibbs_plumbing_matches_reference(kind):
    from pulsar_timing_gibbsspec_amd import PTABlockGibbs, synthetic
    g = golden(f"pta_{kind}.npz")
    gb = PTABlockGibbs(synthetic.array_pta(kind=kind, seed=0), hypersample="conditional",
                       redsample="conditional" if kind == "curn_red" else "mh", seed=1)
    assert gb.param_names == list(g["param_names"])
    assert np.array_equal(np.stack(gb.gwid), g["gwid"])
    assert np.array_equal(gb.get_rho_param_indices(), g["rind"])
    assert np.array_equal(gb.get_hyper_param_indices(), g["hind"])
    assert (gb.rhomin_gw, gb.rhomax_gw) == (float(g["rhomin_gw"]), float(g["rhomax_gw"]))
    assert (gb.rhomin_red, gb.rhomax_red) == (float(g["rhomin_red"]), float(g["rhomax_red"]))


def test_uniform_bounds_and_vector_map():
    from pulsar_timing_gibbsspec_amd.plumbing import expand_names, uniform_bounds, vector_to_dict
    from pulsar_timing_gibbsspec_amd.synthetic import Uniform
    assert uniform_bounds(Uniform("a_rho", -9.0, -4.0, size=3)) == (-9.0, -4.0)
    assert uniform_bounds("x:Uniform(pmin=0.1, pmax=5)") == (0.1, 5.0)
    with pytest.raises(ValueError):
        uniform_bounds("x:Normal(mu=0, sigma=1)")
    ps = [Uniform("a", 0, 1), Uniform("b", 0, 1, size=3), Uniform("c", 0, 1, size=1)]
    assert expand_names(ps) == ["a", "b_0", "b_1", "b_2", "c_0"]
    d = vector_to_dict(ps, np.arange(5.0))
    assert d["a"] == 0.0 and np.array_equal(d["b"], [1.0, 2.0, 3.0]) and d["c"] == 4.0
    assert isinstance(d["c"], float)                   # size-1 vector -> float, as the reference


def test_seed_none_draws_fresh_entropy():
    """seed=None: independent runs get different Philox keys (the reference's unseeded
    global np.random never repeats); the drawn seed is kept for reproduction."""
    from pulsar_timing_gibbsspec_amd.pulsar_gibbs import resolve_seed
    a, b = resolve_seed(None), resolve_seed(None)
    assert a != b
    assert resolve_seed(a[0]) == a and resolve_seed(5) == resolve_seed(5)


def test_indep_array_and_pulsar_sharding():
    from pulsar_timing_gibbsspec_amd import PulsarArrayGibbs, synthetic
    from pulsar_timing_gibbsspec_amd.array_gibbs import balanced_blocks, shard_pulsars
    g = golden("indep_array.npz")
    ptas = synthetic.pulsar_ptas(synthetic.array_pta(kind="indep", seed=0))
    assert [p.pulsars[0] for p in ptas] == list(g["pulsars"])
    m = np.array([p.get_basis()[0].shape[1] for p in ptas])
    assert len(ptas) == 45 and m.min() == 68 and m.max() == 77
    for k, p in enumerate(g["picks"]):
        assert ptas[p].param_names == list(g[f"p{k}_param_names"])
    arr = PulsarArrayGibbs(ptas, nchains=2, seed=3)
    assert arr.pulsars == list(g["pulsars"])
    assert all(np.array_equal(s.gwid, np.arange(60)) for s in arr.samplers)
    for world in (1, 2, 4, 8):
        blocks = [shard_pulsars(ptas, r, world) for r in range(world)]
        assert blocks[0][0] == 0 and blocks[-1][1] == 45
        assert all(a[1] == b[0] and a[0] < a[1] for a, b in zip(blocks, blocks[1:] + [(45, 46)]))
        w = [np.sum(m[lo:hi].astype(float) ** 3) for lo, hi in blocks]
        assert max(w) <= np.sum(m.astype(float) ** 3) / world + (m.max() ** 3)
    assert balanced_blocks([1.0] * 4, 4) == [(0, 1), (1, 2), (2, 3), (3, 4)]


def test_pulsar_array_gibbs_rejects_non_free_spectrum_pulsars():
    """PulsarArrayGibbs fuses every pulsar into one free-spectrum sweep: a pulsar with a white-noise
    (or red / ECORR) Metropolis block is refused up front, not by a shape error mid-run."""
    import pytest
    from pulsar_timing_gibbsspec_amd import synthetic
    from pulsar_timing_gibbsspec_amd.array_gibbs import PulsarArrayGibbs
    ok = synthetic.pulsar_ptas(synthetic.array_pta(kind="indep", seed=0))[:2]
    PulsarArrayGibbs(ok, seed=1)                      # no GPU touched: the context is lazy
    white = synthetic.single_pulsar_pta("J1713+0747", seed=0, efac_vary=True, n_backends=3)
    with pytest.raises(NotImplementedError, match="free-spectrum-only"):
        PulsarArrayGibbs([ok[0], white], seed=1)
