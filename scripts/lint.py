#!/usr/bin/env python3
"""``make lint``: static checks of the Python tree and the HIP sources.

Runs ``ruff check`` and ``mypy`` (configured in pyproject.toml, reference
``pyproject.toml:53-94`` / ``Makefile:1-15``) when they are installed, and ALWAYS runs a built-in
checker that needs nothing beyond the standard library, so the target means something in the
offline MI355X image too:

* every ``.py`` file compiles;
* no unused imports (AST: an imported name never referenced in its module, outside ``__init__``
  re-export modules and names listed in ``__all__``);
* no line over 130 (Python) / 140 (HIP, C++) characters, no trailing whitespace, no tab indentation;
* HIP sources: no CUDA compatibility layers (``__HIP_PLATFORM_*`` dual paths, ``cuda_runtime``
  includes, hipify markers) — the kernels are written for gfx950 directly;
* environment knobs: every ``LLMTRAIN_*`` / ``LLMT_*`` variable read in ``llmtrain/``, ``csrc/`` or
  ``bench.py`` is listed in ``llmtrain/runtime/knobs.py`` (at most ``MAX_KNOBS``), none is read
  from C++, and the knob table of ``docs/debugging.md`` lists exactly those.

Exit status 1 when anything is found (the findings are printed as ``path:line: message``).
"""

from __future__ import annotations

import ast
import importlib.util
import re
import shutil
import subprocess
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
PY_DIRS = ("llmtrain", "tests", "bench", "scripts", "examples")
PY_FILES = ("bench.py", "__graft_entry__.py")
MAX_LINE = 130  # Python
MAX_LINE_NATIVE = 140  # HIP / C++
HIP_FORBIDDEN = (
    (re.compile(r"__HIP_PLATFORM_(AMD|NVIDIA|NVCC)__"), "platform dual path"),
    (re.compile(r"#\s*include\s*[<\"]cuda"), "CUDA header"),
    (re.compile(r"HIPIFY|hipify", re.IGNORECASE), "hipify output"),
)


def python_files() -> list[Path]:
    files = [ROOT / f for f in PY_FILES if (ROOT / f).exists()]
    for d in PY_DIRS:
        files += sorted((ROOT / d).rglob("*.py"))
    return [f for f in files if "build" not in f.parts and ".cache" not in f.parts]


class _Names(ast.NodeVisitor):
    def __init__(self) -> None:
        self.used: set[str] = set()

    def visit_Name(self, node: ast.Name) -> None:
        self.used.add(node.id)

    def visit_Attribute(self, node: ast.Attribute) -> None:
        root = node
        while isinstance(root, ast.Attribute):
            root = root.value  # type: ignore[assignment]
        if isinstance(root, ast.Name):
            self.used.add(root.id)
        self.generic_visit(node)


def _string_names(tree: ast.AST) -> set[str]:
    """Names mentioned in string annotations / __all__ entries (``"torch.Tensor"``)."""
    out: set[str] = set()
    for node in ast.walk(tree):
        if isinstance(node, ast.Constant) and isinstance(node.value, str):
            out.update(re.findall(r"[A-Za-z_][A-Za-z0-9_]*", node.value))
    return out


def check_python(path: Path) -> list[str]:
    rel = path.relative_to(ROOT)
    text = path.read_text()
    findings: list[str] = []
    try:
        tree = ast.parse(text, filename=str(path))
        compile(text, str(path), "exec")
    except SyntaxError as exc:
        return [f"{rel}:{exc.lineno}: syntax error: {exc.msg}"]
    for i, line in enumerate(text.splitlines(), 1):
        if len(line) > MAX_LINE:
            findings.append(f"{rel}:{i}: line too long ({len(line)} > {MAX_LINE})")
        if line.rstrip() != line:
            findings.append(f"{rel}:{i}: trailing whitespace")
        if line.startswith("\t"):
            findings.append(f"{rel}:{i}: tab indentation")
    if path.name == "__init__.py":
        return findings  # re-export modules
    names = _Names()
    names.visit(tree)
    used = names.used | _string_names(tree)
    for node in ast.walk(tree):
        if isinstance(node, (ast.Import, ast.ImportFrom)):
            if isinstance(node, ast.ImportFrom) and node.module == "__future__":
                continue
            for alias in node.names:
                bound = (alias.asname or alias.name).split(".")[0]
                if alias.name == "*" or bound in used:
                    continue
                line = text.splitlines()[node.lineno - 1]
                if "noqa" in line:
                    continue
                findings.append(f"{rel}:{node.lineno}: unused import '{alias.asname or alias.name}'")
    return findings


def check_hip(path: Path) -> list[str]:
    rel = path.relative_to(ROOT)
    findings = []
    for i, line in enumerate(path.read_text().splitlines(), 1):
        for pattern, what in HIP_FORBIDDEN:
            if pattern.search(line):
                findings.append(f"{rel}:{i}: {what} in a gfx950 kernel source")
        if len(line) > MAX_LINE_NATIVE:
            findings.append(f"{rel}:{i}: line too long ({len(line)} > {MAX_LINE_NATIVE})")
    return findings


KNOB_READ = re.compile(r"""(?:environ(?:\.get)?\(|environ\[|getenv\()\s*["'](LLMT[A-Z0-9_]*)""")


def _knob_registry() -> tuple[dict[str, object], int]:
    """KNOBS / MAX_KNOBS of llmtrain/runtime/knobs.py, read without importing the package (torch)."""
    ns: dict[str, object] = {}
    exec(compile((ROOT / "llmtrain" / "runtime" / "knobs.py").read_text(), "knobs.py", "exec"), ns)
    return ns["KNOBS"], ns["MAX_KNOBS"]  # type: ignore[return-value]


def check_knobs() -> list[str]:
    knobs, cap = _knob_registry()
    findings = []
    if len(knobs) > cap:
        findings.append(f"llmtrain/runtime/knobs.py: {len(knobs)} knobs > {cap}")
    files = sorted((ROOT / "llmtrain").rglob("*.py")) + [ROOT / "bench.py"]
    files += [f for f in sorted((ROOT / "csrc").glob("*")) if f.suffix in (".hip", ".h", ".cpp")]
    for f in files:
        rel = f.relative_to(ROOT)
        for i, line in enumerate(f.read_text().splitlines(), 1):
            if f.suffix != ".py" and "getenv" in line:
                findings.append(f"{rel}:{i}: environment read in native code (knobs live in Python)")
            for name in KNOB_READ.findall(line):
                if name not in knobs:
                    findings.append(f"{rel}:{i}: knob {name} is not in llmtrain/runtime/knobs.py")
    documented = set(re.findall(r"^\| `(LLMTRAIN_[A-Z0-9_]+)` \|", (ROOT / "docs" / "debugging.md").read_text(), re.M))
    if documented != set(knobs):
        findings.append(f"docs/debugging.md: knob table {sorted(documented)} != knobs.py {sorted(knobs)}")
    return findings


def run_external() -> int:
    rc = 0
    if shutil.which("ruff") or importlib.util.find_spec("ruff"):
        rc |= subprocess.call([sys.executable, "-m", "ruff", "check", *PY_DIRS, *PY_FILES], cwd=ROOT)
    else:
        print("lint: ruff not installed; built-in checks only")
    if importlib.util.find_spec("mypy"):
        rc |= subprocess.call([sys.executable, "-m", "mypy", "--config-file=pyproject.toml", "llmtrain"], cwd=ROOT)
    else:
        print("lint: mypy not installed; built-in checks only")
    return rc


def main() -> int:
    findings: list[str] = []
    for f in python_files():
        findings += check_python(f)
    for f in sorted((ROOT / "csrc").glob("*")) + sorted((ROOT / "bench" / "native").glob("*.cpp")):
        if f.suffix in (".hip", ".h", ".cpp"):
            findings += check_hip(f)
    findings += check_knobs()
    for line in findings:
        print(line)
    external = run_external() if "--builtin-only" not in sys.argv else 0
    print(f"lint: {len(findings)} finding(s) from the built-in checker")
    return 1 if findings or external else 0


if __name__ == "__main__":
    sys.exit(main())
