"""The CPU oracle under AddressSanitizer + UBSan (the verdict's missing
sanitizer build).  `make -C oracle asan` builds oracle/fuzz_main.c with the
LZ4 and Zstd decoders of the oracle; the run decodes oracle-encoded LZ4 blocks
and the golden libzstd frames plus thousands of truncated / bit-flipped
variants into exact-size heap buffers, so any out-of-bounds read or write, or
undefined behaviour, aborts it.  Host code only (GPU sanitizers are not
available on this pool)."""
import json
import os
import struct
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_oracle_decoders_under_asan_ubsan(tmp_path):
    r = subprocess.run(["make", "-C", os.path.join(ROOT, "oracle"), "asan"], capture_output=True, text=True)
    if r.returncode != 0:
        pytest.skip("no sanitizer toolchain: " + r.stderr[-300:])
    gdir = os.path.join(ROOT, "tests", "golden")
    g = json.load(open(os.path.join(gdir, "zstd_golden.json")))
    blob = open(os.path.join(gdir, g["bin"]), "rb").read()
    recs = bytearray()
    for f in g["frames"]:
        if f["size"] <= (1 << 20):
            fr = blob[f["off"]:f["off"] + f["csize"]]
            recs += struct.pack("<II", len(fr), f["size"]) + fr
    for e in g["corpus"][:600]:
        src = bytes.fromhex(e["src"])
        recs += struct.pack("<II", len(src), max(e["cap"], 0)) + src
    path = tmp_path / "zframes.bin"
    path.write_bytes(bytes(recs))
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=1", UBSAN_OPTIONS="print_stacktrace=1")
    r = subprocess.run([os.path.join(ROOT, "oracle", "_build", "oracle_fuzz_asan"), "600", str(path)],
                       capture_output=True, text=True, env=env, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    assert "sanitized oracle run" in r.stdout
