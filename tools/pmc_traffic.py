"""Per-launch HBM traffic of a kernel from rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes.

Corrections (MI355X_MICROARCH.md §HBM): FETCH_SIZE and WRITE_SIZE are in KiB;
on gfx950 FETCH_SIZE reports 1/2 of the bytes of wide coalesced streaming reads
(x2 here; our reads are 8/16-byte per-lane loads, so this is an upper estimate of
the read side); WRITE_SIZE is exact for 16-B/lane stores.
Writes profiles/<tag>/pmc_traffic.json (bench.py reports it as roofline.traffic).

    python tools/pmc_traffic.py gpurun_out/prof_r01 [kernel_substring] [out.json]

SWEEPS / CHAINS (env, default 100 / 4096) record the launch shape the counts
belong to; bench.py only reports the figure for the same shape.
"""
import csv
import glob
import json
import os
import sys


def per_dispatch(d, counter, kernel, grid=None, first=None):
    """Counter values of the kernel's dispatches in dispatch order; with grid, only launches
    of that many work-items (the headline: CHAINS x 64), and with first, only the first ones
    of those (bench.py runs the headline first: warmup + K/S timed launches; the host-stream
    lines after it share the grid but record elsewhere, and configs[2]'s launches differ)."""
    files = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    rows = []
    for f in files:
        for row in csv.DictReader(open(f)):
            if kernel in row.get("Kernel_Name", "") and row.get("Counter_Name") == counter:
                if grid is None or int(row.get("Grid_Size", -1)) == grid:
                    rows.append((int(row.get("Dispatch_Id", 0)), float(row["Counter_Value"])))
    rows.sort()
    vals = [v for _, v in rows]
    return vals[:first] if first else vals


def main():
    d = sys.argv[1]
    kernel = sys.argv[2] if len(sys.argv) > 2 else "k_sweep_freespec"
    out = sys.argv[3] if len(sys.argv) > 3 else os.path.join(d, "pmc_traffic.json")
    # GRID (work-items per launch) when it is not one wavefront per chain (k_bdraw_tiled: 4 chain
    # groups of 4 waves per workgroup)
    grid = int(os.environ["GRID"]) if "GRID" in os.environ else int(os.environ.get("CHAINS", "4096")) * 64
    first = int(os.environ.get("HEAD_LAUNCHES", "6"))      # 1 warmup + 5 timed (bench defaults)
    fetch = per_dispatch(os.path.join(d, "pmc_fetch"), "FETCH_SIZE", kernel, grid, first)
    write = per_dispatch(os.path.join(d, "pmc_write"), "WRITE_SIZE", kernel, grid, first)
    # the timed launches are the full-size ones (warmup launches may be shorter)
    res = {"kernel": kernel, "n_fetch": len(fetch), "n_write": len(write),
           "sweeps_per_launch": int(os.environ.get("SWEEPS", "100")),
           "chains": int(os.environ.get("CHAINS", "4096"))}
    if fetch and write:
        f = max(fetch)
        w = max(write)
        res.update(fetch_kib=f, write_kib=w, read_bytes=2 * f * 1024, write_bytes=w * 1024,
                   bytes_per_launch=2 * f * 1024 + w * 1024,
                   note="FETCH_SIZE x2 (gfx950 wide-read correction), KiB -> bytes; largest of the headline's "
                        "launches (grid CHAINS x 64, first HEAD_LAUNCHES dispatches)")
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
