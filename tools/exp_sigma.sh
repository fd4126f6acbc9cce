cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/sig
for sg in 3 6 10 16 24; do
  SVGD_MEDIAN_SIGMA=$sg timeout -k 10 120 python bench.py --config cfg5 --steps 20 --warmup 3 --no-cpu > gpurun_out/sig/s$sg.log 2>&1 || exit 1
  echo "sigma $sg $(tail -1 gpurun_out/sig/s$sg.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["phases_ms_per_step"])')"
done
