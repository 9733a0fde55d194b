bash scripts/gpurun_r04_full.sh; rc=$?; [ $rc -le 1 ] || exit $rc
timeout -k 10 300 python tools/miss_profile.py c3 40 > gpurun_out/miss_c3.jsonl 2> gpurun_out/miss_c3.err &&
timeout -k 10 400 python tools/miss_profile.py c5 40 > gpurun_out/miss_c5.jsonl 2> gpurun_out/miss_c5.err &&
BENCH_ARGS="--config c5" bash scripts/gpurun_r04_ab.sh BASE=1 PMX_RED_TAIL=1 &&
mv gpurun_out/ab.jsonl gpurun_out/ab_c5.jsonl &&
BENCH_ARGS="--config c4" bash scripts/gpurun_r04_ab.sh BASE=1 && mv gpurun_out/ab.jsonl gpurun_out/ab_c4.jsonl
