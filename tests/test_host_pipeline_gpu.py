"""Host batch path (capi.hip run_batch): many chunks pipelined over two
streams.  A child process with a 16 MiB staging chunk pushes ~60 blocks
through several chunks per call, mixed sizes and codecs; every result must
match a single-chunk run and the CPU oracle (LZ4 and Zstd level-1 bytes exact,
both round trips)."""
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CHILD = r'''
import hashlib, sys
sys.path.insert(0, sys.argv[1])
from juicefs_amd import compress as C
from juicefs_amd.blockgen import gen_block
from tests import oracle_ctypes
o = oracle_ctypes.Oracle(sys.argv[2])
sizes = [(64 << 10) + 37 * i if i % 3 else (3 << 20) + 1001 * i for i in range(60)]
srcs = [gen_block("TZR"[i % 3] if i % 5 else "T", 4000 + i, n) for i, n in enumerate(sizes)]
lz, zs = C.LZ4(), C.ZStandard()
for c in (lz, zs):
    pairs = [(bytearray(c.CompressBound(len(s))), s) for s in srcs]
    res = c.CompressBatch(pairs)
    frames = []
    for (d, s), (n, e) in zip(pairs, res):
        assert e is None and n > 0, e
        frames.append(bytes(d[:n]))
        if c is lz:
            m, ref = o.lz4_compress(s)
            assert bytes(d[:n]) == ref
        else:  # byte-identical to libzstd 1.4.9 level 1 (the restatement the oracle pins)
            assert bytes(d[:n]) == o.zstd_compress_l1(s)
    outs = [bytearray(len(s)) for s in srcs]
    back = c.DecompressBatch(list(zip(outs, frames)))
    for s, b, (n, e) in zip(srcs, outs, back):
        assert e is None and n == len(s) and bytes(b) == s
print("OK", len(srcs))
'''


def test_multi_chunk_pipeline(gpu, oracle):
    env = dict(os.environ, JFS_HOST_CHUNK_MB="16")
    so = os.path.join(ROOT, "oracle", "_build", "liboracle.so")
    r = subprocess.run([sys.executable, "-c", CHILD, ROOT, so], env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0 and "OK 60" in r.stdout, (r.stdout[-2000:], r.stderr[-2000:])
