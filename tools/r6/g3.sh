# round-6 GPU job 3: decode-batch attention FX=2 (bench + bits), option tests, set A/B
export TMPDIR=/tmp
mkdir -p gpurun_out
for a in "128 405" "64 405" "16 100" "128 30" "100 405"; do timeout -k 10 120 ./tools/micro/dx_bench $a 10 >> gpurun_out/g3_dx.txt 2>&1 || exit 1; done
cat gpurun_out/g3_dx.txt
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_stream.py "tests/test_gpu_full.py::test_full_option_matches_default" "tests/test_gpu_full.py::test_full_fx_seq_one_launch_bit_identical" > gpurun_out/g3_t.log 2>&1 || { tail -30 gpurun_out/g3_t.log; exit 2; }
tail -2 gpurun_out/g3_t.log
for o in "skinny_wdef=1" "skinny_wdef=1,fx_seq=2" "skinny_wdef=1" "skinny_wdef=1,fx_seq=2"; do
  OPT="$o" timeout -k 10 200 python -u tools/r6/set_run.py >> gpurun_out/g3_set.txt 2>&1 || exit 3
done
for o in "skinny_wdef=1" "skinny_wdef=1,refill_group=32,live_prefix=1" "skinny_wdef=1,refill_group=16,live_prefix=1" "skinny_wdef=1,live_prefix=1"; do
  N_UTT=125 SLOTS=63 OPT="$o" timeout -k 10 200 python -u tools/r6/set_run.py >> gpurun_out/g3_share.txt 2>&1 || exit 4
done
