# MFMA counters of the encoder / prefill kernels at 64 x 30 s (the
# encoder_roofline at batch with pmc_mfma showing it): kernel-trace stats + one MFMA PMC
# pass over qasr-bench per config, tools/prof_report.py -> gpurun_out/r5enc/<cfg>/summary.json
export TMPDIR=/tmp
ENC="gemm_kernel|gemm_glds|gemm8p|gemm_q8|enc_attn|prefill_attn|conv1"
for cfg in f16 q8; do
    Q=""; [ "$cfg" = q8 ] && Q="--q8"
    D=gpurun_out/r5enc/$cfg; mkdir -p $D
    timeout -k 10 180 rocprofv3 --kernel-trace --stats -f csv -d $D/stats -o run -- ./qwen3-asr.cpp_amd/qasr-bench $Q --batch 64 --seconds 30 --steps 1 --warmup 1 --tok-rate 0.05 > $D/stats.log 2>&1 || { tail -5 $D/stats.log; exit 1; }
    timeout -k 10 180 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_MOPS_F16 SQ_INSTS_VALU_MFMA_MOPS_F32 SQ_INSTS_VALU_MFMA_MOPS_I8 GRBM_GUI_ACTIVE --kernel-include-regex "$ENC" -f csv -d $D/mfma -o run -- ./qwen3-asr.cpp_amd/qasr-bench $Q --batch 64 --seconds 30 --steps 1 --warmup 0 --tok-rate 0.05 > $D/mfma.log 2>&1 || { tail -5 $D/mfma.log; exit 1; }
    python3 tools/prof_report.py $D > $D/summary.json
    python3 -c "
import json; d=json.load(open('$D/summary.json'))
for k in d['kernels']:
    if 'mfma_util' in k: print('$cfg', k['name'][:60], k['calls'], k['avg_us'], k['mfma_util'], k.get('mfma_tflops'))"
done
