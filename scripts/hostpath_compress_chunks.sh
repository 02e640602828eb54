cd "$GRAFT_REPO_ROOT"
for cfg in "" "JFS_HOST_CHUNK_MB_LZ4C=2048" "JFS_HOST_CHUNK_MB_LZ4C=1024" "JFS_HOST_CHUNK_MB_LZ4C=1024 JFS_LZ4E_SEG_MAX=128"; do
  env $cfg timeout -k 10 200 python scripts/hostpath.py 1024 > gpurun_out/hpc.json || exit 1
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(repr(sys.argv[2]), round(d['lz4_decompress']['value'],2), round(d['lz4_compress']['value'],2), flush=True)" gpurun_out/hpc.json "$cfg"
done
