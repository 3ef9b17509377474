set -eu
export TMPDIR=/tmp
A="--no-cpu-baseline --no-extras --steps 10 --warmup 2"
for L in main q64; do
  lib=fast-slam_amd/lib/libfs2_$L.so; [ $L = main ] && lib=fast-slam_amd/lib/libfs2.so
  FS2_LIB=$lib timeout -k 10 180 rocprofv3 --pmc TA_TA_BUSY_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum GRBM_GUI_ACTIVE --kernel-include-regex "k_candidates" -d gpurun_out/pmcq_ta_$L -o ta --output-format csv -- python3 bench.py $A > gpurun_out/pmcq_ta_$L.log 2>&1
  FS2_LIB=$lib timeout -k 10 180 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS --kernel-include-regex "k_candidates" -d gpurun_out/pmcq_sq_$L -o sq --output-format csv -- python3 bench.py $A > gpurun_out/pmcq_sq_$L.log 2>&1
done
