"""Per-kernel register use of the built library (occupancy guard).

Reads the gfx950 code objects embedded in libpulsar_gibbs.so (.hip_fatbin: one offload bundle
per translation unit), unbundles each with clang-offload-bundler and parses the AMDHSA kernel
metadata from `llvm-readelf --notes`.  CPU only (no GPU needed).

    python tools/kernel_resources.py [lib.so] [name-substring ...]
"""
import os
import re
import subprocess
import sys
import tempfile

LLVM = "/opt/rocm/lib/llvm/bin"
MAGIC = b"__CLANG_OFFLOAD_BUNDLE__"
TARGET = "hipv4-amdgcn-amd-amdhsa--gfx950"


def kernel_resources(lib):
    """{mangled kernel name: {vgpr_count, vgpr_spill_count, sgpr_count, sgpr_spill_count, ...}}"""
    out = {}
    with tempfile.TemporaryDirectory() as d:
        fat = os.path.join(d, "fat.bin")
        subprocess.run([f"{LLVM}/llvm-objcopy", "--dump-section", f".hip_fatbin={fat}", lib, os.path.join(d, "x")],
                       check=True, capture_output=True)
        data = open(fat, "rb").read()
        starts = [m.start() for m in re.finditer(re.escape(MAGIC), data)]
        for i, s in enumerate(starts):
            part = os.path.join(d, f"b{i}.bin")
            open(part, "wb").write(data[s:starts[i + 1] if i + 1 < len(starts) else len(data)])
            co = os.path.join(d, f"b{i}.o")
            r = subprocess.run([f"{LLVM}/clang-offload-bundler", "--unbundle", "--type=o", f"--input={part}",
                                f"--targets={TARGET}", f"--output={co}"], capture_output=True)
            if r.returncode != 0 or not os.path.exists(co) or os.path.getsize(co) == 0:
                continue
            notes = subprocess.run([f"{LLVM}/llvm-readelf", "--notes", co], check=True,
                                   capture_output=True, text=True).stdout
            cur = None
            for line in notes.splitlines():
                m = re.match(r"\s+\.name:\s+(\S+)", line)
                if m:
                    cur = out.setdefault(m.group(1), {})
                    continue
                m = re.match(r"\s+\.(vgpr_count|vgpr_spill_count|sgpr_count|sgpr_spill_count|"
                             r"agpr_count|group_segment_fixed_size|private_segment_fixed_size):\s+(\d+)", line)
                if m and cur is not None:
                    cur[m.group(1)] = int(m.group(2))
    return out


def waves_per_simd(vgprs):
    """Occupancy limit of a kernel's VGPR count (512 per SIMD lane, granule 8)."""
    g = max(8, -(-vgprs // 8) * 8)
    return min(8, 512 // g)


if __name__ == "__main__":
    lib = sys.argv[1] if len(sys.argv) > 1 else os.path.join(
        os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "pulsar_timing_gibbsspec_amd",
        "libpulsar_gibbs.so")
    pats = sys.argv[2:]
    for name, r in sorted(kernel_resources(lib).items()):
        if pats and not any(p in name for p in pats):
            continue
        v = r.get("vgpr_count", 0)
        print(f"{v:4d} vgpr ({waves_per_simd(v)}/SIMD) {r.get('vgpr_spill_count', 0):3d} spill "
              f"{r.get('sgpr_count', 0):4d} sgpr {r.get('sgpr_spill_count', 0):3d} sspill  {name}")
