cd /root/repo && export TMPDIR=/tmp && mkdir -p gpurun_out && rm -rf gpurun_out/pmc_rb* &&
timeout -k 10 200 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES --kernel-trace -d gpurun_out/pmc_rb1 -o run --output-format csv -- ./tools/voc_bench > gpurun_out/pmc_rb1.log 2>&1 &&
timeout -k 10 200 rocprofv3 --pmc SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_MFMA SQ_WAIT_INST_LDS TCP_TOTAL_CACHE_ACCESSES_sum --kernel-trace -d gpurun_out/pmc_rb2 -o run --output-format csv -- ./tools/voc_bench > gpurun_out/pmc_rb2.log 2>&1
