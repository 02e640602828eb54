cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
for c in 2048 4096 8192; do JFS_HOST_CHUNK_MB_LZ4C=$c timeout -k 10 200 python scripts/host_c.py 1024 2>&1 | grep -v amdgpu || exit 1; done
