"""HBM traffic of one configs[3] Zstd decode launch (every jfs::zstdd kernel
of the launch summed) from two rocprofv3 --pmc passes (FETCH_SIZE, WRITE_SIZE;
KiB per dispatch), with the gfx950 FETCH_SIZE correction of MI355X_MICROARCH.md.
usage: traffic_zstd.py <fetch.csv> <write.csv> <blocks> <block_bytes> [out.json]"""
import csv
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def per_kernel(path, counter):
    """{kernel short name: KiB per decode launch} for jfs::zstdd kernels: the
    sum over the profiled run's dispatches divided by its number of launches
    (zexec_kernel runs once per launch)"""
    d, launches = {}, set()
    for r in csv.DictReader(open(path)):
        k = r["Kernel_Name"]
        if "zstdd::" not in k or r["Counter_Name"] != counter:
            continue
        name = k.split("zstdd::")[1].split("(")[0]
        d[name] = d.get(name, 0.0) + float(r["Counter_Value"])
        if name == "zexec_kernel":
            launches.add(r["Dispatch_Id"])
    if not d or not launches:
        raise SystemExit(f"no jfs::zstdd {counter} rows in {path}")
    return {k: v / len(launches) for k, v in d.items()}, len(launches)


fpath, wpath, nblk, bb = sys.argv[1], sys.argv[2], int(sys.argv[3]), int(sys.argv[4])
(f, nf), (w, nw) = per_kernel(fpath, "FETCH_SIZE"), per_kernel(wpath, "WRITE_SIZE")
fk, wk = sum(f.values()), sum(w.values())
out = {
    "blocks": nblk, "block_bytes": bb, "kernels": "every jfs::zstdd kernel of one jfs_zstd_decompress_device launch",
    "launches_profiled": [nf, nw],
    "fetch_size_kb": fk, "write_size_kb": wk,
    "per_kernel_kb": {k: {"fetch": f.get(k, 0.0), "write": w.get(k, 0.0)} for k in sorted(set(f) | set(w))},
    "hbm_bytes_raw": (fk + wk) * 1024.0,
    "hbm_bytes_per_launch": (2.0 * fk + wk) * 1024.0,
    "correction": "MI355X_MICROARCH.md: on gfx950 FETCH_SIZE reads 1/2 of wide coalesced stream bytes -> "
                  "hbm = (2*FETCH_SIZE + WRITE_SIZE)*1024; exact only for 16-B streaming loads, so the true "
                  "traffic lies between hbm_bytes_raw and hbm_bytes_per_launch",
    "source": f"rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE, separate passes ({fpath}, {wpath})",
}
from bench import kernel_src_sha256, ZSTD_KERNEL_SOURCES  # noqa: E402
out["kernel_src_sha256"] = kernel_src_sha256(ZSTD_KERNEL_SOURCES)
try:
    out["git_head"] = subprocess.run(["git", "-C", ROOT, "rev-parse", "HEAD"], capture_output=True,
                                     text=True).stdout.strip() or None
except Exception:
    out["git_head"] = None
s = json.dumps(out, indent=1)
print(s)
if len(sys.argv) > 5:
    open(sys.argv[5], "w").write(s + "\n")
