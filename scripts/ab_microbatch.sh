cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/mb
for r in 1 2; do for mb in 128 192 256; do
  timeout -k 10 300 python bench.py --steps 12 --warmup 3 --micro-batch $mb > gpurun_out/mb/mb${mb}_r${r}.log 2>&1 || { echo "mb$mb failed"; tail -5 gpurun_out/mb/mb${mb}_r${r}.log; exit 1; }
  echo "mb$mb r$r: $(tail -1 gpurun_out/mb/mb${mb}_r${r}.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["peak_mem_gib"], d["final_loss"])')"
done; done
