#!/bin/bash
# summarize a gpu_session.sh run from gpurun_out/
cd "$(dirname "$0")/.."
grep rc gpurun_out/steps.log 2>/dev/null
for f in smoke pytest_gpu pytest_gpu_all; do [ -f gpurun_out/$f.log ] && tail -2 gpurun_out/$f.log; done
for f in bench bench_direct; do
  [ -f gpurun_out/$f.log ] && tail -1 gpurun_out/$f.log | python -c "import json,sys
try:
  d=json.loads(sys.stdin.read()); r=d['roofline']
  print(d['config']['mode'], '%.3e QP/s' % d['value'], 'ms/step %.4f' % d['ms_per_step'], 'kernel %s us %.1f' % (r['kernel'], r['avg_launch_us']), 'frac %.3f' % r['frac'], 'cpu', d.get('cpu_baseline', {}).get('value'))
except Exception as e: print('bench parse failed', e)"
done
[ -f gpurun_out/prof/run_kernel_stats.csv ] && cut -d, -f1-4 gpurun_out/prof/run_kernel_stats.csv | cut -c1-120
