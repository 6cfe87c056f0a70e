"""Per-draw SQ instruction counts of the headline kernel from one rocprofv3 --pmc pass
(run_counter_collection.csv) -> profiles/sq_headline.json (read by bench.py's simd_issue).

    python tools/sq_summary.py gpurun_out/r06l/sq/run_counter_collection.csv k_sweep_pair \
        --chains 4096 --sweeps 100 --source "..." [--out profiles/sq_headline.json]

Per dispatch the counter values are summed over the rows rocprofv3 writes for it; per launch = the mean
over the kernel's dispatches; per draw = per launch / (chains x sweeps).
"""
import argparse
import collections
import csv
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("csv")
    ap.add_argument("kernel", help="kernel-name fragment")
    ap.add_argument("--chains", type=int, default=4096)
    ap.add_argument("--sweeps", type=int, default=100)
    ap.add_argument("--source", default="")
    ap.add_argument("--out", default=os.path.join(ROOT, "profiles", "sq_headline.json"))
    a = ap.parse_args()
    per = collections.defaultdict(lambda: collections.defaultdict(float))
    name = None
    for r in csv.DictReader(open(a.csv)):
        if a.kernel not in r["Kernel_Name"]:
            continue
        name = r["Kernel_Name"]
        per[int(r["Dispatch_Id"])][r["Counter_Name"]] += float(r["Counter_Value"])
    if not per:
        raise SystemExit(f"no dispatch of {a.kernel} in {a.csv}")
    counters = sorted({c for d in per.values() for c in d})
    launch = {c: sum(d[c] for d in per.values()) / len(per) for c in counters}
    draws = a.chains * a.sweeps
    from __graft_entry__ import source_hash
    out = {"kernel": name.split("::")[-1], "chains": a.chains, "sweeps_per_launch": a.sweeps, "dispatches": len(per),
           "per_draw": {c: v / draws for c, v in launch.items() if c != "SQ_WAVES"},
           "per_launch": launch, "library_sources": source_hash(), "source": a.source}
    json.dump(out, open(a.out, "w"), indent=1)
    print(json.dumps(out["per_draw"], indent=1))


if __name__ == "__main__":
    main()
