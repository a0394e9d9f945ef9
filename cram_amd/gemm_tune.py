"""Pinned GEMM solutions for the IE sweep's projection shapes, through PyTorch TunableOp's results file.

hipBLASLt's heuristic pick for the sweep's q/k/v (N = 6144) and o_proj (N = 4096, K = 4096) GEMMs at
M = 33 x T rows is 9-12 % slower than the best solution TunableOp finds (`tools/tunable_probe.py`, same-process
A/B: 8.86 -> 8.55 ms per Llama-3-8B layer at M = 29184).  Tuning online is not an option (every question has
its own M = 33 x T rounded to 256), so the solutions tuned once are pinned for every M the sweep and the packed
prefill can produce: a TunableOp results file is written at start-up with one line per (N, K, M) and read
back with tuning off.  The decode steps' weight-streaming GEMMs (M = batch rows: 256 for configs 2 / 4, 16 for
config 5) get exact (N, K, M) lines where the tuned pick beat the default by >= 5 % in a same-process probe
(`tools/tune_decode_gemms.py`, `decode_solutions`); they act inside the step graph's capture.  Shapes without a
line (other models, other M) run the default heuristic.

The solution ids belong to one hipBLASLt / rocBLAS build: the file carries the validators of the build they
were tuned on (`data/gemm_solutions.json`), and nothing is pinned when the running build differs.

Scope: TunableOp is a process-wide switch, so it is only turned on inside `pinned()` blocks — the engine's
sweep and packed prefill — and restored to the caller's state on exit; other GEMMs of the process (the
transformers model of the drop-in path, user code) keep torch's default selection and TunableOp settings.
"""
from __future__ import annotations

import contextlib
import json
import os
import tempfile
from typing import Dict, Iterable, Tuple

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SOLUTIONS = os.path.join(REPO, "data", "gemm_solutions.json")
_installed = None
_tried = None
_decode_rows = frozenset()   # M values that have decode-step lines
_scope = None                # "sweep" inside pinned(), "decode" inside pinned(decode=True)


def _signature(N: int, K: int, M: int) -> str:
    # F.linear(x [M, K], w [N, K]) is a column-major TN GEMM with m = N, n = M, k = K
    return f"tn_{N}_{M}_{K}_ld_{K}_{K}_{N}"


def load(path: str = SOLUTIONS) -> dict:
    with open(path) as f:
        return json.load(f)


def validators_match(tuned: Dict[str, str]) -> bool:
    try:
        have = {str(v[0]): str(v[1]) for v in torch.cuda.tunable.get_validators()}   # (name, value) pairs
    except (RuntimeError, IndexError, TypeError):
        return False
    return all(have.get(k) == v for k, v in tuned.items())


def install(m_values: Iterable[int], dtype: str = "BFloat16", path: str = SOLUTIONS) -> bool:
    """Pin the tuned solutions for every M in m_values; returns False (nothing pinned) on a different build."""
    global _installed, _decode_rows
    sol = load(path)
    if not validators_match(sol["validators"]):
        return False
    lines = [f"Validator,{k},{v}" for k, v in sol["validators"].items()]
    for key, name in sol["solutions"].items():
        N, K = (int(x) for x in key.split("x"))
        for M in m_values:
            lines.append(f"GemmTunableOp_{dtype}_TN,{_signature(N, K, M)},{name},0")
    for key, name in sol.get("decode_solutions", {}).items():     # decode steps: exact (N, K, M = batch rows)
        N, K, M = (int(x) for x in key.split("x"))
        lines.append(f"GemmTunableOp_{dtype}_TN,{_signature(N, K, M)},{name},0")
    fd, fn = tempfile.mkstemp(prefix="cram_gemm_", suffix=".csv")
    with os.fdopen(fd, "w") as f:
        f.write("\n".join(lines) + "\n")
    tun = torch.cuda.tunable
    prev = (tun.is_enabled(), tun.tuning_is_enabled())
    tun.enable(True)
    tun.tuning_enable(False)
    try:
        ok = tun.read_file(fn)
    finally:
        tun.enable(prev[0])
        tun.tuning_enable(prev[1])
        os.unlink(fn)
    _installed = fn if ok else None
    if ok:
        _decode_rows = frozenset(int(k.split("x")[2]) for k in sol.get("decode_solutions", {}))
    return bool(ok)


@contextlib.contextmanager
def pinned(decode: bool = False):
    """Use the pinned solutions for the GEMMs issued inside the block (TunableOp on, tuning off), then restore
    the process's previous TunableOp state.  A no-op when nothing was pinned (other build, no GPU, A/B off).
    decode=True: the decode step (its exact-M lines act); otherwise the sweep / prefill, where `shadowed(M)` tells
    ops.linear to run a GEMM whose M has a decode line without TunableOp, so decode picks never touch the sweep."""
    global _scope
    if not _tried:
        yield
        return
    tun = torch.cuda.tunable
    prev = (tun.is_enabled(), tun.tuning_is_enabled(), _scope)
    tun.enable(True)
    tun.tuning_enable(False)
    _scope = "decode" if decode else "sweep"
    try:
        yield
    finally:
        tun.enable(prev[0])
        tun.tuning_enable(prev[1])
        _scope = prev[2]


def shadowed(M: int) -> bool:
    """True inside a sweep / prefill pinned() block for a row count that only decode steps may pin."""
    return _scope == "sweep" and M in _decode_rows


@contextlib.contextmanager
def unpinned():
    """TunableOp off for the GEMMs inside the block (restored after)."""
    tun = torch.cuda.tunable
    prev = tun.is_enabled()
    tun.enable(False)
    try:
        yield
    finally:
        tun.enable(prev)


def sweep_rows(lo: int = 8192, hi: int = 65536, step: int = 256) -> Tuple[int, ...]:
    """Row counts the sweep's suffix batches (33 x T, padded_rows) and the packed prefill chunks take: multiples of 256."""
    return tuple(range(lo, hi + 1, step))


def ensure() -> bool:
    """Load the pins once per process (CrAMEngine does this on a GPU; they act inside `pinned()` only); False
    when the build differs."""
    global _tried
    if _tried is None:
        off = os.environ.get("CRAM_GEMM_PIN", "1") == "0"              # A/B switch: default heuristic everywhere
        _tried = install(sweep_rows()) if torch.cuda.is_available() and not off else False
    return _tried


def uninstall() -> None:
    global _tried
    _tried = False
