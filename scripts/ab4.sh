cd $GRAFT_REPO_ROOT
for r in 1 2; do
 for e in "LLMTRAIN_FUSED_GEMM=0" "LLMTRAIN_FGEMM_MAX_A_MB=1024" "LLMTRAIN_FGEMM_MAX_A_MB=1024 LLMT_FGEMM_WAVES_OF_CUS=0"; do
  v=$(env $e timeout -k 10 300 python bench.py --steps 10 --warmup 3 --micro-batch 64 2>/dev/null | python3 -c "import json,sys; print(json.loads(sys.stdin.read())['value'])")
  echo "mb64 [$e]: $v"
 done
done
