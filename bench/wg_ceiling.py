import json, sys, torch
sys.path.insert(0, "bench"); sys.path.insert(0, ".")
from micro import timeit
from llmtrain.ops import _ext
_ext.require()
M = 131072
for name, (N, K) in {"qkv": (2304, 768), "out": (768, 768), "fc": (3072, 768), "proj": (768, 3072), "head": (50257, 768)}.items():
    dy = torch.randn(M, N, device="cuda", dtype=torch.bfloat16)
    x = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
    acc = torch.zeros(N, K, device="cuda")
    dyT = dy.t().contiguous(); xT = x.t().contiguous()
    f = 2.0 * M * N * K
    res = {}
    res["ours"] = timeit(lambda: torch.ops.llmtrain_hip.wgrad_gemm(dy, x, acc, 0, 0), iters=10, warmup=3)
    res["blt_tn_bf16out"] = timeit(lambda: torch.mm(dyT, xT.t()), iters=10, warmup=3)
    res["blt_nt_bf16out"] = timeit(lambda: torch.mm(dy.t(), x), iters=10, warmup=3)
    del dyT, xT
    print(json.dumps({"gemm": name, **{k: [round(v, 3), round(f / v / 1e9, 1)] for k, v in res.items()}}), flush=True)
    del dy, x, acc
    torch.cuda.empty_cache()
