"""Per-launch HBM traffic of the ECORR lines' kernels from round 6's two PMC passes over the same command
(`bench.py --no-cpu-baseline --pta none --config5 0 --indep 0 --steps 2 --warmup 1 --ecorr-steps 2
--ess 0`: FETCH_SIZE in tools/gpu_r06d.sh, WRITE_SIZE in tools/gpu_r06e.sh).  The bench's time-based
warm-up makes the two passes' dispatch ids differ, so each pass's timing runs are found on their own.
Kernels are picked by name and by the bench's
timing loops: the full likelihood launch (`em._eval`, 10 back-to-back k_ecorr_prefix<5, true, PC, false>
dispatches) and the incremental Metropolis step (`ecorr_step_roofline`, k_ecorr_prefix<5, true, false,
true> after its 3 warm-up calls), first for the `ecorr` line (shared operands), then `ecorr_white`
(per-chain operands).  Corrections as tools/pmc_traffic.py: KiB -> bytes, FETCH_SIZE x2 on gfx950.

    python tools/pmc_ecorr_r06.py gpurun_out/r06d/pmc gpurun_out/r06e/wr
"""
import csv
import glob
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def rows(d, counter):
    out = {}
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if r["Counter_Name"] == counter and "k_ecorr_prefix" in r["Kernel_Name"]:
                out[int(r["Dispatch_Id"])] = (r["Kernel_Name"].split("::")[-1].split("(")[0],
                                              float(r["Counter_Value"]))
    return out


def runs(disp, name):
    """Maximal runs of consecutive dispatch ids (step 1) of the kernel ``name``."""
    ids = sorted(i for i, (n, _) in disp.items() if n == name)
    out, cur = [], []
    for i in ids:
        if cur and i != cur[-1] + 1:
            out.append(cur)
            cur = []
        cur.append(i)
    if cur:
        out.append(cur)
    return out


def main():
    fdir, wdir = sys.argv[1], sys.argv[2]
    F, W = rows(fdir, "FETCH_SIZE"), rows(wdir, "WRITE_SIZE")
    # the bench's timing loops are the only back-to-back (>= 10) runs of these kernels
    timed = {("ecorr", "full"): "k_ecorr_prefix<5, true, false, false>",
             ("ecorr_white", "full"): "k_ecorr_prefix<5, true, true, false>",
             ("ecorr", "step"): "k_ecorr_prefix<5, true, false, true>",
             ("ecorr_white", "step"): "k_ecorr_prefix<5, true, false, true>"}
    res = {}
    for (line, what), name in timed.items():
        k = 1 if (what == "step" and line == "ecorr_white") else 0
        sel = []
        for D in (F, W):
            rr = [r for r in runs(D, name) if len(r) >= 10]
            assert len(rr) == (2 if what == "step" else 1), (line, what, [len(r) for r in rr])
            sel.append(rr[k][-10:])
        fk = sum(F[i][1] for i in sel[0]) / len(sel[0])
        wk = sum(W[i][1] for i in sel[1]) / len(sel[1])
        res[(line, what)] = dict(kernel=name, dispatches_fetch=sel[0], dispatches_write=sel[1], fetch_kib=fk,
                                 write_kib=wk,
                                 read_bytes=2 * fk * 1024, write_bytes=wk * 1024,
                                 bytes_per_launch=2 * fk * 1024 + wk * 1024)
    note = ("round 6 PMC passes (tools/gpu_r06d.sh FETCH_SIZE, tools/gpu_r06e.sh WRITE_SIZE) over bench.py's "
            "ECORR lines, the bench's own timing launches; FETCH_SIZE x2 (gfx950 wide-read correction), KiB -> bytes")
    for (line, what), v in res.items():
        name = {("ecorr", "full"): "pmc_traffic_ecorr.json", ("ecorr_white", "full"): "pmc_traffic_ecorr_white.json",
                ("ecorr", "step"): "pmc_traffic_ecorr_step.json",
                ("ecorr_white", "step"): "pmc_traffic_ecorr_white_step.json"}[(line, what)]
        v.update(chains=4096, sweeps_per_launch=1, source="profiles/r06d, profiles/r06e", note=note)
        json.dump(v, open(os.path.join(ROOT, "profiles", name), "w"), indent=1)
        print(name, v["kernel"], "%.1f MB read + %.1f MB written" % (v["read_bytes"] / 1e6, v["write_bytes"] / 1e6))


if __name__ == "__main__":
    main()
