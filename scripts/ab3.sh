cd $GRAFT_REPO_ROOT
for r in 1 2; do
 for cfg in "64 LLMTRAIN_FUSED_GEMM=1" "128 LLMTRAIN_FUSED_GEMM=0" "64 LLMTRAIN_FUSED_GEMM=0"; do set -- $cfg
  v=$(env $2 timeout -k 10 300 python bench.py --steps 10 --warmup 3 --micro-batch $1 2>/dev/null | python3 -c "import json,sys; print(json.loads(sys.stdin.read())['value'])")
  echo "mb$1 $2: $v"
 done
done
