# Bench spread on one box (test tooling): bench.py three times back to back (no CPU baseline,
# no fp32 build), the value / stem times of each run.
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
for r in 1 2 3; do
  timeout -k 10 300 python -u bench.py --no-cpu-baseline --fp32-steps 0 --steps 40 > gpurun_out/rep_$r.log 2>&1 || exit $?
  tail -1 gpurun_out/rep_$r.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('run $r:', d['value'], 'vol/s', d['ms_per_step'], 'ms/step; stem', r['t_fwd_us'], '+', r['t_wgrad_us'], 'us, frac', r['frac'])"
done
