#!/bin/bash
# Round measurement on the GPU box (development tool): the default bench line, a rocprofv3
# kernel-trace/stats pass of the same bench command, and two PMC passes (FETCH_SIZE and
# WRITE_SIZE in separate runs) for the HBM traffic of the dominant kernel class.
# Usage (from the repo root, via gpurun): bash sherpa-vietnamese-asr_amd/tools/profile_round.sh TAG
set -e
TAG=${1:-r}
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/prof_$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 python3 $R/bench.py > $OUT/bench.json 2> $OUT/bench.err
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/stats -o run -- python3 $R/bench.py --no-cpu-baseline --steps 3 --warmup 1 > $OUT/stats_bench.json 2> $OUT/stats.err
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/pmc_fetch -o run -- python3 $R/bench.py --no-cpu-baseline --steps 1 --warmup 1 > $OUT/pmc_fetch.log 2>&1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/pmc_write -o run -- python3 $R/bench.py --no-cpu-baseline --steps 1 --warmup 1 > $OUT/pmc_write.log 2>&1
timeout -k 10 300 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d $OUT/pmc_mfma -o run -- python3 $R/bench.py --no-cpu-baseline --steps 1 --warmup 1 > $OUT/pmc_mfma.log 2>&1
for st in campp vad; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/stats_$st -o run -- python3 $R/bench.py --stage $st --no-cpu-baseline --steps 3 --warmup 1 > $OUT/stats_$st.json 2> $OUT/stats_$st.err
done
echo done
