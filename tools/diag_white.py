"""Diagnostic (GPU): where does the white-noise path's first b draw lose accuracy?"""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch
from oracle import gibbs_oracle as O
from tests.conftest import golden
from tests.parity_data import normwise_rel, white_params, white_replay
from pulsar_timing_gibbsspec_amd import _lib
from pulsar_timing_gibbsspec_amd.white import WhiteNoiseModel

g = golden("white_mh_j1713.npz")
rp = white_replay(g)
ctx = _lib.Context(0, seed=5)
T = g["T"]; m = T.shape[1]; gwid = np.asarray(g["gwid"]); gw = rp["gwind"]
wm = WhiteNoiseModel(ctx, [T], [g["r"]], [g["sigma"]], [g["backends"]], [gwid], [np.full(m - gwid.size, 1e-40)],
                     [white_params(g)], 1)
x0 = g["x0"]
xd = torch.as_tensor(x0[None].copy(), device=ctx.device)
wm.refresh(xd, x0.size)
TNTd, dd = wm.tnt_host(0, 0)
N = rp["N_of"](x0)
TNT, d = O.tnt(T, N, g["r"])
A = np.abs(T).T / N @ np.abs(T)
print("TNT err / (eps*|T||T|/N):", np.max(np.abs(TNTd - TNT) / (A * 2.2e-16)), " d rel", normwise_rel(dd, d))
order = O.chol_order(m, gwid)
ph = np.full(m, 1e-40); ph[gwid] = 1 / np.repeat(10 ** (2 * x0[gw]), 2)
bo = O.bdraw_chol(TNT, d, ph, rp["z0"], order)
bod = O.bdraw_chol(TNTd, dd, ph, rp["z0"], order)
print("oracle(numpy TNT) vs ref", normwise_rel(bo, rp["b_first"]), " oracle(GPU TNT) vs oracle(numpy TNT)", normwise_rel(bod, bo))
phF = torch.as_tensor(ph[gwid][None].copy(), device=ctx.device)
b = torch.zeros(1, wm.ldb, dtype=torch.float64, device=ctx.device)
info = torch.zeros(1, dtype=torch.int32, device=ctx.device)
z = np.zeros((1, wm.ldb)); z[0, :m] = rp["z0"]
wm.bdraw(phF, b, info, z=torch.as_tensor(z, device=ctx.device))
bg = b[0, :m].cpu().numpy()
print("GPU vs oracle(GPU TNT)", normwise_rel(bg, bod), " GPU vs ref", normwise_rel(bg, rp["b_first"]), "info", int(info[0]))
# the prefix on the host from the GPU TNT
pf = O.prefix_factor(TNTd, dd, gwid, np.full(m - gwid.size, 1e-40))
bp = O.bdraw_prefix(pf, ph[gwid], rp["z0"])
print("host prefix draw (GPU TNT) vs oracle(GPU TNT)", normwise_rel(bp, bod), " GPU vs host prefix draw", normwise_rel(bg, bp))
mod = wm.model[:wm.mstride].cpu().numpy()
NF = gwid.size
S0d = mod[:NF * (NF + 1)].reshape(NF, NF + 1)[:, :NF]
dFd = mod[NF * (NF + 1):NF * (NF + 1) + NF]
print("S0 rel err", np.max(np.abs(S0d - pf["S0"])) / np.max(np.abs(pf["S0"])), " dF rel", normwise_rel(dFd, pf["dF"]))
ev = np.linalg.eigvalsh(pf["S0"] + np.diag(ph[gwid]))
print("cond S", ev.max() / ev.min())
