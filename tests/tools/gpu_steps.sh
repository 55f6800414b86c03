# Run GPU steps in order, each under its own time limit; stop at the first failure (test
# tooling).  Usage: bash tests/tools/gpu_steps.sh TAG 'cmd1' 'cmd2' ...   Output per step in
# gpurun_out/TAG_<i>.log; the last line of each log is echoed.
TAG=$1; shift
export TMPDIR=/tmp
mkdir -p gpurun_out
i=0
for c in "$@"; do
  i=$((i + 1))
  timeout -k 10 300 bash -c "$c" > gpurun_out/${TAG}_$i.log 2>&1
  rc=$?
  echo "[$i rc=$rc] $c"; tail -3 gpurun_out/${TAG}_$i.log | cut -c1-400
  if [ $rc -ne 0 ]; then exit $rc; fi
done
