"""Decode a few golden Zstd frames on the GPU and print codes (debug aid)."""
import json, os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np, torch
from juicefs_amd import device as D
from tests.oracle_ctypes import Oracle
g = json.load(open(os.path.join(ROOT, "tests/golden/zstd_golden.json")))
blob = open(os.path.join(ROOT, "tests/golden", g["bin"]), "rb").read()
orc = Oracle(os.path.join(ROOT, "oracle/_build/liboracle.so"))
sel = sys.argv[1] if len(sys.argv) > 1 else "12"
ents = g["frames"][:int(sel)] if sel.isdigit() else [f for f in g["frames"] if f"{f['cls']}{f['level']}_{f['size']}" == sel]
dev = torch.device("cuda:0")
for f in ents:
    c = blob[f["off"]:f["off"] + f["csize"]]
    src = torch.from_numpy(np.frombuffer(c, dtype=np.uint8).copy()).to(dev)
    out = torch.zeros(f["size"] + 64, dtype=torch.uint8, device=dev)
    desc = D.make_desc(src, [0], [len(c)], out, [0], [f["size"]])
    ret = torch.zeros(1, dtype=torch.int32, device=dev)
    D.zstd_decompress(desc, ret)
    torch.cuda.synchronize()
    r = int(ret.item())
    n, ref = orc.zstd_decompress(c, f["size"])
    got = out[:max(r, 0)].cpu().numpy().tobytes()
    first = next((i for i in range(min(len(got), len(ref))) if got[i] != ref[i]), None)
    print(f["cls"], f["level"], f["size"], "gpu", r, "oracle", n, "match", got == ref, "first_diff", first, flush=True)
