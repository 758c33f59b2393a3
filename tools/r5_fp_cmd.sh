set -o pipefail
cd /root/repo && mkdir -p gpurun_out/r5/fp && export TMPDIR=/tmp
timeout -k 10 200 ./tools/fused_probe > gpurun_out/r5/fp/fused_probe.json 2> gpurun_out/r5/fp/err.txt || exit $?
for pass in a b; do
  if [ $pass = a ]; then C="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU"; else C="SQ_BUSY_CYCLES SQ_ACTIVE_INST_ANY SQ_INST_CYCLES_VMEM SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE GRBM_COUNT"; fi
  timeout -s KILL 120 rocprofv3 --pmc $C --output-format csv -d gpurun_out/r5/fp/sq_$pass -o run -- ./tools/fused_probe fused_t16_np3_nb6_fix4 > gpurun_out/r5/fp/sq_$pass.out 2>&1 || exit $?
done
echo done
