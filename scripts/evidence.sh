#!/bin/bash
# Round evidence on the GPU box (run from the repo root under gpurun):
#   GPU parity tests, smoke, PMC traffic of the headline kernel (stamped),
#   the full bench line (with that traffic), rocprofv3 kernel stats of the
#   headline and of the Zstd decode, HBM bytes of the Zstd decode kernels.
#   Every step has its own time limit; the script stops at the first failure.
#   Bulky profiler output stays under /tmp; summaries go to gpurun_out/ev/.
set -e
export TMPDIR=/tmp
O=gpurun_out/ev
T=/tmp/ev
mkdir -p $O $T
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1
tail -1 $O/gpu_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
tail -1 $O/smoke.log
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $T/pf -o pf --output-format csv -- python scripts/prof_run.py 4096 1 T > $O/pf.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $T/pw -o pw --output-format csv -- python scripts/prof_run.py 4096 1 T > $O/pw.log 2>&1
# instruction mix (VALU / SALU / LDS per token, wait share) of the headline and Zstd decode kernels
SQC="SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_INSTS_VMEM"
JFS_NOVERIFY=1 timeout -s KILL 120 rocprofv3 --pmc $SQC -d $T/pi -o pi --output-format csv -- python scripts/prof_run.py 4096 1 T > $O/pi.log 2>&1
python scripts/pmc_summary.py $(find $T/pi -name '*counter_collection.csv' | head -1) --kernel lz4_decode > $O/pmc_lz4_decode.txt
python scripts/traffic.py $(find $T/pf -name '*counter_collection.csv' | head -1) $(find $T/pw -name '*counter_collection.csv' | head -1) lz4_decode_kernel 4096 4194304 $O/traffic.json > /dev/null
# HBM traffic of the Zstd decode kernels (one launch each pass, frames from the cache)
timeout -k 10 300 python scripts/prof_run.py 4096 0 T zstd > /dev/null 2>&1
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $T/zpf -o zpf --output-format csv -- python scripts/prof_run.py 4096 1 T zstd > $O/zpf.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $T/zpw -o zpw --output-format csv -- python scripts/prof_run.py 4096 1 T zstd > $O/zpw.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc $SQC -d $T/zpi -o zpi --output-format csv -- python scripts/prof_run.py 4096 1 T zstd > $O/zpi.log 2>&1
python scripts/pmc_summary.py $(find $T/zpi -name '*counter_collection.csv' | head -1) --kernel z > $O/pmc_zstd_decode.txt
python scripts/traffic_zstd.py $(find $T/zpf -name '*counter_collection.csv' | head -1) $(find $T/zpw -name '*counter_collection.csv' | head -1) 4096 4194304 $O/traffic_zstd.json > /dev/null
timeout -k 10 900 python bench.py --traffic-file $O/traffic.json --zstd-traffic-file $O/traffic_zstd.json > $O/bench.json 2> $O/bench.err
tail -c 400 $O/bench.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $T/kt_lz4 -o kt --output-format csv -- python bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-extras --no-host-path --traffic-file $O/traffic.json > $O/kt_lz4.log 2>&1
find $T/kt_lz4 -name '*kernel_stats.csv' -exec cp {} $O/lz4_kernel_stats.csv \;
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $T/kt_zstd -o kt --output-format csv -- python scripts/prof_run.py 4096 3 T zstd > $O/kt_zstd.log 2>&1
find $T/kt_zstd -name '*kernel_stats.csv' -exec cp {} $O/zstd_kernel_stats.csv \;
du -sh $O
echo evidence-done
