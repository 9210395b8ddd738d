# Stage-model GPU tests, then two SQ / LDS PMC passes of the default bench (tools/pmc_kernels.py reads them)
R=$GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_stage_onnx.py tests/test_gpu_vad.py tests/test_gpu_vibert.py tests/test_gpu_campp.py > gpurun_out/stage_tests.log 2>&1 || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_INSTS_LDS GRBM_GUI_ACTIVE --output-format csv -d $R/gpurun_out/pmcA -o run -- python3 $R/bench.py --no-cpu-baseline --parity-precision none --steps 1 --warmup 1 > $R/gpurun_out/pmcA.log 2>&1 || exit 2
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_LDS_LOAD_BANDWIDTH SQ_INSTS_LDS_STORE_BANDWIDTH SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_WAIT_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE --output-format csv -d $R/gpurun_out/pmcB -o run -- python3 $R/bench.py --no-cpu-baseline --parity-precision none --steps 1 --warmup 1 > $R/gpurun_out/pmcB.log 2>&1 || exit 3
