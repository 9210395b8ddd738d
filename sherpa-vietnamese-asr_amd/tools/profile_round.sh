#!/bin/bash
# Round measurement on the GPU box (development tool): the default bench line, a rocprofv3
# kernel-trace/stats pass of the same bench command, PMC passes (FETCH_SIZE and WRITE_SIZE in
# separate runs, MFMA busy) for the dominant kernel class, kernel stats of the CAM++ / VAD
# stages, and the bench lines of BASELINE configs 3, 4 and 5 (and their token-exact f16x3
# forms).  Profiled passes run with --parity-precision none (the parity line is a child
# process of the bench; it is measured in the plain runs).
# Usage (from the repo root, via gpurun): bash sherpa-vietnamese-asr_amd/tools/profile_round.sh TAG [PART]
# PART 1 / 2 runs the first / second half (each within one gpurun call's limit); default both.
# PART 3: the f16x3 line's PMC passes and config 5 in f16x3.
set -e
TAG=${1:-r}
PART=${2:-all}
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/prof_$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
if [ "$PART" != 2 ] && [ "$PART" != 3 ]; then
timeout -k 10 400 python3 $R/bench.py > $OUT/bench.json 2> $OUT/bench.err
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/stats -o run -- python3 $R/bench.py --no-cpu-baseline --parity-precision none --steps 3 --warmup 1 > $OUT/stats_bench.json 2> $OUT/stats.err
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/pmc_fetch -o run -- python3 $R/bench.py --no-cpu-baseline --parity-precision none --steps 1 --warmup 1 > $OUT/pmc_fetch.log 2>&1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/pmc_write -o run -- python3 $R/bench.py --no-cpu-baseline --parity-precision none --steps 1 --warmup 1 > $OUT/pmc_write.log 2>&1
timeout -k 10 300 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d $OUT/pmc_mfma -o run -- python3 $R/bench.py --no-cpu-baseline --parity-precision none --steps 1 --warmup 1 > $OUT/pmc_mfma.log 2>&1
for st in campp vad; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/stats_$st -o run -- python3 $R/bench.py --stage $st --no-cpu-baseline --steps 3 --warmup 1 > $OUT/stats_$st.json 2> $OUT/stats_$st.err
done
timeout -k 10 300 python3 $R/bench.py --no-cpu-baseline --method modified_beam_search --beam 8 --hotwords-file default > $OUT/bench_beam8_hotwords.json 2> $OUT/bench_beam8.err
# config 3 on the beam-calibrated weights (beam 8 emits at the greedy rate) and its f16x3 form
timeout -k 10 300 python3 $R/bench.py --no-cpu-baseline --weights beam-calibrated --method modified_beam_search --beam 8 --hotwords-file default > $OUT/bench_beam8_hotwords_beamcal.json 2> $OUT/bench_beam8_beamcal.err
fi
if [ "$PART" != 1 ] && [ "$PART" != 3 ]; then
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/stats_f16x3 -o run -- python3 $R/bench.py --no-cpu-baseline --precision f16x3 --parity-precision none --steps 3 --warmup 1 > $OUT/stats_f16x3.json 2> $OUT/stats_f16x3.err
timeout -k 10 300 python3 $R/bench.py --no-cpu-baseline --precision f16x3 --parity-precision none --method modified_beam_search --beam 8 --hotwords-file default > $OUT/bench_beam8_hotwords_f16x3.json 2> $OUT/bench_beam8_f16x3.err
timeout -k 10 300 python3 $R/bench.py --no-cpu-baseline --weights beam-calibrated --precision f16x3 --parity-precision none --method modified_beam_search --beam 8 --hotwords-file default > $OUT/bench_beam8_hotwords_f16x3_beamcal.json 2> $OUT/bench_beam8_f16x3_beamcal.err
timeout -k 10 300 python3 $R/bench.py --stage rover --steps 4 --warmup 1 --hotwords-file default > $OUT/bench_rover.json 2> $OUT/bench_rover.err
timeout -k 10 300 python3 $R/bench.py --stage pipe --steps 4 --warmup 1 > $OUT/bench_pipe.json 2> $OUT/bench_pipe.err
timeout -k 10 300 python3 $R/bench.py --stage campp > $OUT/bench_campp.json 2> $OUT/bench_campp.err
timeout -k 10 300 python3 $R/bench.py --stage vad > $OUT/bench_vad.json 2> $OUT/bench_vad.err
timeout -k 10 300 python3 $R/bench.py --stage dropin --steps 3 --warmup 1 --hotwords-file default > $OUT/bench_dropin.json 2> $OUT/bench_dropin.err
timeout -k 10 300 python3 $R/bench.py --stage dropin --precision bf16 --steps 3 --warmup 1 --hotwords-file default > $OUT/bench_dropin_bf16.json 2> $OUT/bench_dropin_bf16.err
# DESIGN §9's single-GPU proxies of the 8-rank shard plan (largest LPT share of the hour)
timeout -k 10 300 python3 $R/bench.py --no-cpu-baseline --parity-precision none --proxy-ranks 8 > $OUT/bench_proxy8.json 2> $OUT/bench_proxy8.err
timeout -k 10 300 python3 $R/bench.py --stage rover --steps 4 --warmup 1 --hotwords-file default --no-cpu-baseline --proxy-ranks 8 > $OUT/bench_rover_proxy8.json 2> $OUT/bench_rover_proxy8.err
fi
if [ "$PART" = 3 ]; then
# the token-exact f16x3 line's PMC passes (HBM bytes, MFMA busy) and config 5 in f16x3
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/pmc_f16x3_fetch -o run -- python3 $R/bench.py --no-cpu-baseline --precision f16x3 --parity-precision none --no-sub-lines --steps 1 --warmup 1 > $OUT/pmc_f16x3_fetch.log 2>&1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/pmc_f16x3_write -o run -- python3 $R/bench.py --no-cpu-baseline --precision f16x3 --parity-precision none --no-sub-lines --steps 1 --warmup 1 > $OUT/pmc_f16x3_write.log 2>&1
timeout -k 10 300 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d $OUT/pmc_f16x3_mfma -o run -- python3 $R/bench.py --no-cpu-baseline --precision f16x3 --parity-precision none --no-sub-lines --steps 1 --warmup 1 > $OUT/pmc_f16x3_mfma.log 2>&1
timeout -k 10 300 python3 $R/bench.py --stage pipe --precision f16x3 --steps 4 --warmup 1 > $OUT/bench_pipe_f16x3.json 2> $OUT/bench_pipe_f16x3.err
fi
echo done
