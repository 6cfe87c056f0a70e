"""Copy a GPU check's outputs (gpurun_out/<tag>) into profiles/<tag> for the record: the rocprofv3
kernel stats, the bench JSON lines, pytest / smoke tails, and launch_stats.log with each kernel's
per-launch list cut to its first 60 launches (the full trace stays in gpurun_out).
    python tools/save_profile.py r04f"""
import os
import shutil
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
KEEP = ("bench.json", "bench_prof.json", "bench.err", "kernel_stats.csv", "pytest.txt", "smoke.log",
        "indep_parity.json", "prof.err")


def main(tag):
    src, dst = os.path.join(ROOT, "gpurun_out", tag), os.path.join(ROOT, "profiles", tag)
    os.makedirs(dst, exist_ok=True)
    for f in KEEP:
        if os.path.exists(os.path.join(src, f)):
            shutil.copy(os.path.join(src, f), os.path.join(dst, f))
    ls = os.path.join(src, "launch_stats.log")
    if os.path.exists(ls):
        out = []
        for line in open(ls):
            if " launches, ms: " in line:
                head, vals = line.rstrip("\n").split(" launches, ms: ")
                v = vals.split()
                line = f"{head} launches, ms: {' '.join(v[:60])}{' ...' if len(v) > 60 else ''}\n"
            out.append(line)
        open(os.path.join(dst, "launch_stats.log"), "w").writelines(out)
    print("saved", dst, sorted(os.listdir(dst)))


if __name__ == "__main__":
    main(sys.argv[1])
