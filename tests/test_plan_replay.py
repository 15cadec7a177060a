"""The factorisation plans libptzba builds (ptzba_plan_export, host only), replayed task by task on the CPU
(tests/chol_plan_exec.py restates k_chol_step's tile tasks in numpy) on an SPD matrix with the reduced camera
system's coupling structure, must reproduce numpy's Cholesky factor: the one- and two-level nested orders, the
delayed trailing updates and their 2 x 2 trailing blocks.  Plan logic only: the device arithmetic is checked by
the GPU tests (test_gpu_nested2.py, test_gpu_config4.py)."""
import os

import numpy as np
import pytest

from conftest import ROOT

import chol_plan_exec as cpe
import ptzba


def band_window(n, w):
    return np.minimum(np.arange(n) + w, n - 1).astype(np.int32)


CASES = {
    "config3": lambda: np.load(os.path.join(ROOT, "tests", "golden", "config3_window.npy")),
    "band300": lambda: band_window(300, 24),
}


@pytest.mark.parametrize("env", [{}, {"PTZBA_ND_DEPTH": "1"}, {"PTZBA_CHOL_DELAY": "2"},
                                 {"PTZBA_CHOL_DELAY": "2", "PTZBA_CHOL_BLOCKS": "0"},
                                 {"PTZBA_CHOL_DELAY": "2", "PTZBA_ND_DEPTH": "1"}])
@pytest.mark.parametrize("case", sorted(CASES))
def test_plan_replays_to_the_cholesky_factor(monkeypatch, case, env):
    for k in ("PTZBA_ND_DEPTH", "PTZBA_CHOL_DELAY", "PTZBA_CHOL_BLOCKS"):
        monkeypatch.delenv(k, raising=False)
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    win = CASES[case]()
    pos, tasks, off, n_aug, _ = ptzba.plan_export(win, 1)
    ld = (n_aug + 1 + 31) // 32 * 32
    S = cpe.test_matrix(pos, win, n_aug, ld)
    Lf, _ = cpe.replay(S, tasks, off)
    Lref = np.linalg.cholesky(S)
    assert np.abs(Lf - Lref).max() <= 1e-12 * np.abs(Lref).max()
    if env == {"PTZBA_CHOL_DELAY": "2", "PTZBA_ND_DEPTH": "1"}:
        assert ((tasks[:, 0] & 3) == 3).any()  # the delayed plan uses 2 x 2 trailing blocks
    if env.get("PTZBA_CHOL_BLOCKS") == "0":
        assert not ((tasks[:, 0] & 3) == 3).any()
