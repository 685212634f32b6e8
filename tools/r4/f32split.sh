# aligner prefill scores as split fp16 (var_f32split.so) vs fp32 MFMA: aligner leg time, classes vs the default
export TMPDIR=/tmp
mkdir -p gpurun_out
for L in qwen3-asr.cpp_amd/libqasr.so qwen3-asr.cpp_amd/var_f32split.so; do
QASR_LIB_OVERRIDE=$L timeout -k 10 300 python -u tools/r4/align_time.py 2>&1 | tail -2
done
QASR_VARIANT=qwen3-asr.cpp_amd/var_f32split.so timeout -k 10 600 python -u tools/r4/px_check.py || exit 1
exit 0
