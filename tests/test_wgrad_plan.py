"""Weight-gradient split planner (csrc/gemm_wgrad_pp.hip ``plan_pp``), through the catch-all
``wgrad_pp_plan`` op: no GPU work, so it runs on the CPU wherever the extension loads.

The plan is a fixed function of the shape (deterministic runs depend on that), GPT-2 124M shapes
keep the square 256 x 256 tiling, and GPT-2 XL's d = 1600 shapes take the strip / swapped tiling
(docs/round6.md §10)."""

from __future__ import annotations

import pytest
import torch

from llmtrain.ops import _ext

pytestmark = pytest.mark.skipif(not _ext.load(), reason="HIP extension not built")

KEYS = ("swap", "tiles", "split", "chunk", "mode", "nwg", "s_tiles", "s_split", "s_chunk", "s_mode", "s_nwg", "ns")


def plan(M, N, K, lda=None, bias=False, split=0, mode=0):
    out = torch.ops.llmtrain_hip.wgrad_pp_plan(M, N, K, lda or N, K, bias, split, mode)
    return dict(zip(KEYS, out))


@pytest.mark.parametrize("N,K", [(2304, 768), (768, 768), (3072, 768), (768, 3072), (50257, 768)])
def test_gpt2_124m_shapes_keep_square_tiles(N, K):
    p = plan(131072, N, K, lda=50304 if N == 50257 else N)
    assert p["swap"] == 0 and p["s_tiles"] == 0 and p["s_nwg"] == 0
    assert p["nwg"] == p["tiles"] * p["split"]
    assert p["split"] == 1 or p["chunk"] * p["split"] >= 131072


@pytest.mark.parametrize("N,K,swap", [(4800, 1600, 0), (6400, 1600, 0), (1600, 6400, 1)])
def test_gpt2_xl_shapes_take_the_tail_tiling(N, K, swap):
    p = plan(32768, N, K)
    sq = plan(32768, N, K, mode=8)
    assert p["swap"] == swap
    assert p["s_tiles"] > 0 and p["s_nwg"] == p["s_tiles"] * p["s_split"]
    # the strips cover the 64-column tail: 512-wide n strips over the long side
    long_side = K if swap else N
    assert p["s_tiles"] == -(-long_side // 512)
    assert p["ns"] < 0.9 * sq["ns"]  # taken only with a >= 10 % modelled margin
    assert sq["swap"] == 0 and sq["s_tiles"] == 0


def test_square_out_projection_stays_square():
    # 1600 x 1600 measured slower with strips (docs/round6.md §10): below the planner's margin
    p = plan(32768, 1600, 1600)
    assert p["s_tiles"] == 0 and p["swap"] == 0


def test_plan_is_a_fixed_function_of_the_shape():
    for args in [(32768, 4800, 1600), (32768, 1600, 6400), (131072, 2304, 768), (16384, 50257, 1600, 50304)]:
        first = plan(*args)
        for _ in range(3):
            assert plan(*args) == first


def test_swap_needs_a_dense_dy_for_the_bias_pass():
    # a column slice of dY (lda > N) cannot feed the separate column-sum pass: no swap with a bias
    assert plan(4096, 320, 2304, lda=384, bias=True)["swap"] == 0
    assert plan(4096, 320, 2304, lda=384, bias=False)["swap"] == 1


def test_forced_splits_are_honoured():
    p = plan(32768, 4800, 1600, split=2 + 65536 * 5)
    assert p["split"] == 2 and p["s_split"] == 5
