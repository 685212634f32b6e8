# round-6 GPU job 13: prefill_attn_exact4_kernel with the DPP wait states (px_bench, every case) and the fmaxf-scan form
mkdir -p gpurun_out
for b in px_bench_ px_bench_dpx4_scan0; do
  echo "== $b"
  timeout -k 10 120 ./tools/micro/$b 4 || exit 1
done
