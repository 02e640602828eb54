# Diagnostic: needs the diag variant (scripts/build_variant.sh diag -DJFS_DIAG; JFS_GPU_LIB=juicefs_amd/lib/libjfsgpu_diag.so)
import ctypes, sys
sys.path.insert(0, '/root/repo')
import torch
from juicefs_amd import _lib
lib = _lib.load()
out = torch.zeros(128, dtype=torch.int32, device='cuda')
lib.jfs_selftest_lds_align.argtypes = [ctypes.c_void_p]
print('rc', lib.jfs_selftest_lds_align(out.data_ptr()))
o = out.cpu().numpy().view('uint32')
ok128 = all(o[l*4+j] == int.from_bytes(bytes([(l + 4*j + t) & 255 for t in range(4)]), 'little') for l in range(16) for j in range(4))
ok64 = all(o[64+l*2+j] == int.from_bytes(bytes([(4*l + 4*j + t) & 255 for t in range(4)]), 'little') for l in range(16) for j in range(2))
print('b128 unaligned ok', ok128, 'b64 4-aligned ok', ok64)
print([hex(x) for x in o[:16]])
