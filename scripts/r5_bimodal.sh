# five back-to-back driver commands (no CPU baseline): ms/step, pairs and the
# per-iteration levels / window verdicts / full searches of the timed iterations
set -e
for i in 1 2 3 4 5; do
  timeout -k 10 120 python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/r5_bi_$i.json 2> gpurun_out/r5_bi_$i.err
  python -c "
import json;d=json.load(open('gpurun_out/r5_bi_$i.json'));t=d['timed_iterations']
print($i,round(d['ms_per_step'],5),round(d['compute_roofline']['pairs_evaluated_per_launch']),round(d['roofline']['avg_launch_ms'],5),round(d['whole_icp']['ms_per_iteration'],5))
print('  levels',t['levels']);print('  window',t['window']);print('  full',t['full_searches'])"
done
