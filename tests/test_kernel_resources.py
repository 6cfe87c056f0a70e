"""Occupancy guard for the hot kernels (CPU: reads the built library's code-object metadata).

The tile b-draw and the fused sweep are f64-issue bound at a fixed number of waves per SIMD;
a change that pushes a kernel past a VGPR boundary silently costs 25-30 % (k_bdraw at NF = 60:
164 -> 170 VGPRs, 3 -> 2 waves/SIMD, CURN sweep 0.71 -> 0.89 ms on MI355X, round 2).
"""
import os

import pytest

from tools.kernel_resources import kernel_resources, waves_per_simd

LIB = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "pulsar_timing_gibbsspec_amd",
                   "libpulsar_gibbs.so")


@pytest.fixture(scope="module")
def res():
    if not os.path.exists(LIB):
        pytest.skip("library not built")
    return kernel_resources(LIB)


def one(res, frag):
    hits = [r for n, r in res.items() if frag in n]
    assert len(hits) == 1, (frag, [n for n in res if frag in n])
    return hits[0]


# (mangled-name fragment, minimum waves per SIMD, VGPR spills allowed)
HOT = [
    ("k_bdrawILi60ELi0ELi4ELi3E", 3, 2),           # PTA / CURN b|rho (configs[3]); 4 chain groups
                                                   # per workgroup: 2 spills, measured faster (r03h)
    ("k_bdraw_tiledILi60ELi0ELi4ELb1ELb0E", 3, 0),  # PTA b|rho on register-tile model copies (nm <= 16)
    ("k_bdraw_tiledILi60ELi0ELi4ELb0ELb0E", 3, 0),  # ... nm > 16 (configs[3]: row-major fixed block)
    ("k_bdraw_tiledILi60ELi0ELi4ELb1ELb1E", 3, 0),  # ... with the red MH block's lnL_p (round 4)
    ("k_bdraw_tiledILi60ELi0ELi4ELb0ELb1E", 3, 0),
    ("k_lnlike_margILi60ELi0ELi4EE", 3, 0),         # lnL_p fill of shut gates / full seed
    ("k_sweep_freespec_rmILi60ELi0ELi4ELi3E", 3, 16),  # configs[2] (nm up to 17)
    ("k_sweep_freespecILi60ELi0ELi4ELi3E", 3, 16),
    ("k_sweep_freespecILi60ELi0ELi12ELi3E", 3, 40),    # 12-wave hand-off workgroups (the headline's
    ("k_sweep_freespec_rmILi60ELi0ELi12ELi3E", 3, 40),  # 4096 chains): 38 spills outside the body  # headline fused sweep (configs[1], [2]): 3 waves,
                                                    # 13 spills outside the inner body (round 3)
    ("k_bdraw_pairILi4EE", 2, 2),                  # PTA b draw, two chains per wave (opt-in, round 6;
                                                   # 1 spill with the look-ahead factorisation)
    ("k_sweep_pairILi4EE", 2, 12),                 # two chains per wave (the headline since round 6):
                                                   # both chains' tiles at 2 waves/SIMD, 10 spills
                                                   # outside the draw
    ("k_rho_red_waveE", 4, 0),                     # CURN + red grid CDF (f64 wave kernel)
    ("k_rho_red_certE", 4, 0),                     # CURN + red grid CDF (round-3 certified f32)
    ("k_rho_red_cert16E", 3, 0),                   # ... the default since round 4 (16 lanes per row)
    ("k_rho_curn_fastILi5EE", 3, 0),               # 0.60 -> 0.53 ms at 3 waves/SIMD (round 3); CF_K = 5
    ("k_rho_curn_fastILi4EE", 3, 0),               # (configs[3]'s 45 pulsars) and 4, coefficients via LDS
    ("k_rho_curn_sum_waveILi16EE", 2, 0),
    ("k_white_syrkILi14EE", 2, 0),                 # configs[4] per-chain TNT (m = 216)
    ("k_tntEPK", 4, 0),                            # TNT / d, compensated block sums
    ("k_ecorr_prefixILi5ELb1ELb0ELb0E", 3, 4),     # ECORR likelihood, shared chunks (round 5:
                                                   # 3 waves/SIMD with 3 spills, 5 % faster than 2)
    ("k_ecorr_prefixILi5ELb1ELb1ELb0E", 2, 0),     # ... per-chain operands (white noise sampled)
    ("k_ecorr_prefixILi5ELb1ELb0ELb1E", 2, 0),     # ... incremental Metropolis step
]


@pytest.mark.parametrize("frag,min_waves,spills", HOT)
def test_hot_kernel_occupancy(res, frag, min_waves, spills):
    r = one(res, frag)
    assert waves_per_simd(r["vgpr_count"]) >= min_waves, (frag, r)
    assert r.get("vgpr_spill_count", 0) <= spills, (frag, r)


def test_every_kernel_has_metadata(res):
    assert len(res) > 50
    assert all("vgpr_count" in r for r in res.values())
