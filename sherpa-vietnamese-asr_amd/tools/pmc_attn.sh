# Two SQ / LDS PMC passes and a kernel trace of the default bench (tools/pmc_kernels.py reads
# the counter CSVs; argument: output tag)
R=$GRAFT_REPO_ROOT
T=${1:-pmc}
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_INSTS_LDS GRBM_GUI_ACTIVE --output-format csv -d $R/gpurun_out/${T}A -o run -- python3 $R/bench.py --no-cpu-baseline --parity-precision none --steps 1 --warmup 1 > $R/gpurun_out/${T}A.log 2>&1 || exit 2
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_LDS_LOAD_BANDWIDTH SQ_INSTS_LDS_STORE_BANDWIDTH SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_WAIT_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE --output-format csv -d $R/gpurun_out/${T}B -o run -- python3 $R/bench.py --no-cpu-baseline --parity-precision none --steps 1 --warmup 1 > $R/gpurun_out/${T}B.log 2>&1 || exit 3
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/${T}T -o run -- python3 $R/bench.py --no-cpu-baseline --parity-precision none --steps 1 --warmup 1 > $R/gpurun_out/${T}T.log 2>&1 || exit 4
