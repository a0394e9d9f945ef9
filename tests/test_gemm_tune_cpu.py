"""Host logic of the pinned GEMM solutions (cram_amd/gemm_tune.py): the solutions file parses, decode-step pins are
exact (N, K, M) keys, and they are shadowed inside the sweep / prefill scope only (no GPU needed)."""
import torch

from cram_amd import gemm_tune


def test_solutions_file_parses():
    sol = gemm_tune.load()
    assert set(sol["validators"]) >= {"HIPBLASLT_VERSION", "ROCBLAS_VERSION", "GCN_ARCH_NAME"}
    for key, name in sol["solutions"].items():
        N, K = (int(x) for x in key.split("x"))
        assert N > 0 and K > 0 and name.startswith("Gemm_")
    for key, name in sol.get("decode_solutions", {}).items():
        N, K, M = (int(x) for x in key.split("x"))
        assert M in (16, 256, 512) and name.startswith("Gemm_")   # config 5, round-2 config 2, configs 2 / 4 now
        assert gemm_tune._signature(N, K, M) == f"tn_{N}_{M}_{K}_ld_{K}_{K}_{N}"


class _FakeTunable:
    """Stand-in for torch.cuda.tunable's process switches (the real ones need a device)."""
    def __init__(self):
        self.on, self.tuning = False, True

    def enable(self, v=True):
        self.on = bool(v)

    def is_enabled(self):
        return self.on

    def tuning_enable(self, v=True):
        self.tuning = bool(v)

    def tuning_is_enabled(self):
        return self.tuning


def test_decode_pins_shadowed_only_in_sweep_scope(monkeypatch):
    monkeypatch.setattr(gemm_tune, "_tried", True)
    monkeypatch.setattr(gemm_tune, "_decode_rows", frozenset({16, 256}))
    tun = _FakeTunable()
    monkeypatch.setattr(torch.cuda, "tunable", tun)
    before = (tun.is_enabled(), tun.tuning_is_enabled())
    assert not gemm_tune.shadowed(256)                     # outside any pinned() block
    with gemm_tune.pinned():
        assert gemm_tune.shadowed(256) and gemm_tune.shadowed(16)
        assert not gemm_tune.shadowed(29184)               # the sweep's own pinned row counts act
        with gemm_tune.unpinned():
            assert not tun.is_enabled()
        assert tun.is_enabled() and not tun.tuning_is_enabled()
    with gemm_tune.pinned(decode=True):
        assert not gemm_tune.shadowed(256)                 # decode steps use their pins
    assert (tun.is_enabled(), tun.tuning_is_enabled()) == before
    assert gemm_tune._scope is None
