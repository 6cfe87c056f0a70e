"""tools/pmc_traffic.py picks the headline's own launches (grid CHAINS x 64, first
HEAD_LAUNCHES dispatches) out of a whole-bench PMC pass (CPU; synthetic counter CSVs)."""
import csv
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _write(path, counter, rows):
    os.makedirs(path, exist_ok=True)
    with open(os.path.join(path, "run_counter_collection.csv"), "w", newline="") as fh:
        w = csv.writer(fh)
        w.writerow(["Dispatch_Id", "Grid_Size", "Kernel_Name", "Counter_Name", "Counter_Value"])
        for did, grid, name, val in rows:
            w.writerow([did, grid, name, counter, val])


def test_headline_launches_only(tmp_path):
    k = "void k_sweep_freespec<60, 0, 4, 3>(SweepArgs)"
    head = 4096 * 64
    # warmup (50 sweeps), 5 timed launches, then host-stream launches (same grid, larger
    # writes) and configs[2] launches (other grid, much larger)
    writes = [(1, head, k, 170.0)] + [(2 + i, head, k, 340.0) for i in range(5)] + \
             [(7 + i, head, k, 999.0) for i in range(3)] + [(20, 737280, k, 9999.0)]
    fetch = [(d, g, n, v / 100.0) for d, g, n, v in writes]
    _write(str(tmp_path / "pmc_write"), "WRITE_SIZE", writes)
    _write(str(tmp_path / "pmc_fetch"), "FETCH_SIZE", fetch)
    out = tmp_path / "t.json"
    env = dict(os.environ, CHAINS="4096", HEAD_LAUNCHES="6", SWEEPS="100")
    subprocess.run([sys.executable, os.path.join(ROOT, "tools", "pmc_traffic.py"), str(tmp_path),
                    "k_sweep_freespec", str(out)], check=True, env=env, capture_output=True)
    d = json.load(open(out))
    assert d["n_write"] == 6 and d["write_kib"] == 340.0 and d["fetch_kib"] == 3.4
    assert d["bytes_per_launch"] == 340.0 * 1024 + 2 * 3.4 * 1024
