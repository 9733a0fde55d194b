# the driver command three times back to back (CPU baseline included), with
# the per-iteration evidence of the timed iterations
set -e
for i in 1 2 3; do
  timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r5_drv_$i.json 2> gpurun_out/r5_drv_$i.err
  python -c "
import json;d=json.load(open('gpurun_out/r5_drv_$i.json'));t=d['timed_iterations']
print($i,round(d['ms_per_step'],5),round(d['compute_roofline']['pairs_evaluated_per_launch']),round(d['roofline']['avg_launch_ms'],5),round(d['whole_icp']['ms_per_iteration'],5),d['parity']['pass'])
print('  levels',t['levels']);print('  window',t['window']);print('  full',t['full_searches'])"
done
