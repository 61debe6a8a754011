"""Static checks on the inline GCN assembly in csrc/ (CPU only).

An inline-asm block that runs a scalar ALU instruction which writes SCC (s_add_u32, s_cmp_*,
s_and_b32, ...) must list "scc" among its clobbers: otherwise the compiler may keep a comparison
result in SCC across the block and branch on the overwritten flag.  In round 5 a variant of the
fused GEMM did exactly that — the `++is_s == nst` test before the LDS-DMA block read the carry of
`s_add_u32 m0, m0, 0x400`, so the second K stage re-loaded stage 0 (docs/round5.md §13).
"""

from __future__ import annotations

import re
from pathlib import Path

CSRC = Path(__file__).resolve().parents[1] / "csrc"

# SALU opcodes that write SCC (gfx9 family): arithmetic with carry/overflow, compares, bitwise ops
_SCC_WRITERS = re.compile(
    r"\bs_(add|sub|addc|subb|cmp|cmpk|and|or|xor|andn2|orn2|nand|nor|xnor|not|lshl|lshr|ashr|bfe|"
    r"min|max|abs|absdiff|bitcmp|lshl\d_add)_\w+"
)


def _asm_blocks(text: str):
    for m in re.finditer(r"asm\s+volatile\s*\(", text):
        depth, i = 1, m.end()
        while depth and i < len(text):
            depth += {"(": 1, ")": -1}.get(text[i], 0)
            i += 1
        yield text[m.start():i]


def test_scc_writing_asm_declares_scc_clobber():
    offenders = []
    for src in sorted(CSRC.glob("*.hip")) + sorted(CSRC.glob("*.h")):
        text = src.read_text()
        for block in _asm_blocks(text):
            code = " ".join(re.findall(r'"((?:[^"\\]|\\.)*)"', block))
            if _SCC_WRITERS.search(code) and '"scc"' not in block:
                line = text[: text.index(block)].count("\n") + 1
                offenders.append(f"{src.name}:{line}")
    assert not offenders, f"inline asm writes SCC without an \"scc\" clobber: {offenders}"


def test_lint_sees_the_dma_stage_block():
    # the check above is only worth something if it parses the block that needed the fix
    text = (CSRC / "gemm_fused.hip").read_text()
    blocks = [b for b in _asm_blocks(text) if "s_add_u32 m0" in b]
    assert blocks and all('"scc"' in b for b in blocks)
