"""Host-side checks of the reduced-system plan (api.hip choose_order_plan, through the host-only
ptzba_plan_summary): which system order ptzba_set_problem picks for a coupling window, its elimination
levels and back-substitution chains.  No device is needed.  The numeric equivalence of the orders (the
same Gauss-Newton step and optimum under every order) is checked on the GPU (test_gpu_ba.py,
test_gpu_config3.py)."""
import os

import numpy as np
import pytest

from conftest import ROOT

import ptzba


@pytest.fixture
def nd_env():
    old = os.environ.get("PTZBA_ND_DEPTH")
    yield
    if old is None:
        os.environ.pop("PTZBA_ND_DEPTH", None)
    else:
        os.environ["PTZBA_ND_DEPTH"] = old


def band_window(n, w):
    return np.minimum(np.arange(n) + w, n - 1).astype(np.int32)


def test_config3_two_level_dissection(nd_env):
    """Config 3 (500 KF, coupling window ~95 frames, up to 120): two dissection levels give 26 elimination
    levels and four back-substitution chains of at most 25 tile columns, against 30 levels and chains of 29 with one level."""
    win = np.load(os.path.join(ROOT, "tests", "golden", "config3_window.npy"))
    os.environ.pop("PTZBA_ND_DEPTH", None)
    two = ptzba.plan_summary(win, 1)
    os.environ["PTZBA_ND_DEPTH"] = "1"
    one = ptzba.plan_summary(win, 1)
    assert one["nd_depth"] == 1 and one["levels"] == 30 and one["chains"] == 2 and one["longest_chain"] == 29
    assert two["nd_depth"] == 2 and two["chains"] == 4
    assert two["levels"] == 26 and two["longest_chain"] == 25
    assert two["n_aug"] == one["n_aug"] == 1536
    assert two["bs_steps"] > 0  # the blocked back-solve also has a schedule over the separator tree


def test_order_choice_follows_the_level_count(nd_env):
    os.environ.pop("PTZBA_ND_DEPTH", None)
    # short chain: natural order (no split shortens it)
    s = ptzba.plan_summary(band_window(20, 5), 1)
    assert s["nd_depth"] == 0 and s["chains"] == 1
    # a long uniform band: the two-level order wins and stays a valid plan
    s = ptzba.plan_summary(band_window(800, 60), 1)
    os.environ["PTZBA_ND_DEPTH"] = "1"
    s1 = ptzba.plan_summary(band_window(800, 60), 1)
    assert s["nd_depth"] == 2 and s["levels"] < s1["levels"]
    # natural ordering requested: never dissected
    assert ptzba.plan_summary(band_window(800, 60), 1, ptzba.ORDER_NATURAL)["nd_depth"] == 0


def test_plan_summary_rejects_bad_windows():
    with pytest.raises(ptzba.PtzbaError):
        ptzba.plan_summary(np.array([0, 5, 2], np.int32), 1)  # frame 1 couples past the last frame
    with pytest.raises(ptzba.PtzbaError):
        ptzba.plan_summary(np.array([1, 0, 2], np.int32), 1)  # frame 1's window ends before it


def test_config4_keeps_one_level_with_trailing_blocks(nd_env):
    """Config 4 (5000 KF in 10 tilt rows, coupling window ~560 frames, up to 1114): the two-level order would
    have fewer levels (189 vs 265) but levels of up to 18K tasks; the planner's cost estimate keeps the one-level
    order, with delayed trailing updates in 2 x 2 blocks."""
    os.environ.pop("PTZBA_ND_DEPTH", None)
    win = np.load(os.path.join(ROOT, "tests", "golden", "config4_window.npy"))
    s = ptzba.plan_summary(win, 1)
    assert s["nd_depth"] == 1 and s["levels"] == 265 and s["panel_pairs"] == 2, s
    _, tasks, _, _, _ = ptzba.plan_export(win, 1)
    typ = tasks[:, 0] & 3
    assert (typ == 3).sum() > 50 * (typ == 1).sum()  # nearly every trailing tile rides in a block


def test_dist_form_choice_never_predicts_a_slowdown(nd_env):
    """Round 6: bench.py --gpus N picks the form of the sharded solve with the smaller predicted
    trial (ptzba.choose_dist_form, api.hip ptzba_dist_form_estimate: slowest rank's factorisation estimate + its
    collectives as ring all-reduces).  Config 3's rank tree does not shorten the chain (its separators are dense ~110
    frames), so from 4 ranks on its extra exchanges lose to the replicated solve; config 4's tree factorisation is
    ~1.3x shorter than the whole system's and its exchanges are a fraction of the packed system, so it keeps the tree.
    The chosen form's estimate is never above the other's, and at config 3 never above the single-GPU factorisation
    plus the replicated collectives."""
    os.environ.pop("PTZBA_ND_DEPTH", None)
    w3 = np.load(os.path.join(ROOT, "tests", "golden", "config3_window.npy"))
    w4 = np.load(os.path.join(ROOT, "tests", "golden", "config4_window.npy"))
    expect3 = {2: "tree", 4: "replicated", 8: "replicated"}
    for n, form in expect3.items():
        f, e = ptzba.choose_dist_form(w3, n)
        assert f == form, (n, e)
        chosen = e["tree_us"] if f == "tree" else e["replicated_us"]
        other = e["replicated_us"] if f == "tree" else e["tree_us"]
        assert other is None or chosen <= other
        assert e["replicated_doubles"] > e["tree_doubles"] > 0
    for n in (2, 4, 8):
        f, e = ptzba.choose_dist_form(w4, n)
        assert f == "tree" and e["tree_factorisation_us"] < e["full_factorisation_us"], (n, e)
    assert ptzba.choose_dist_form(w3, 1) == ("single", None)
    # a larger alpha moves config 3 at N = 2 to the form with fewer collectives per trial
    e2 = ptzba.dist_form_estimate(w3, 2, alpha_us=200.0)
    assert e2["tree_collectives"] >= 2


def test_replicated_shards_cover_every_landmark_in_contiguous_blocks():
    """The replicated form's landmark -> rank map: contiguous blocks of ~equal record counts, -1 only for landmarks
    without records."""
    rng = np.random.default_rng(0)
    n_lm = 1000
    lm = rng.integers(0, n_lm - 10, 50000)  # the last ten landmarks have no records
    for world in (2, 3, 8):
        own = ptzba.replicated_shards(lm, n_lm, world)
        assert (own[-10:] == -1).all() and (own[:n_lm - 10] >= 0).all()
        live = own[own >= 0]
        assert (np.diff(live) >= 0).all() and set(live.tolist()) == set(range(world))
        counts = np.bincount(own[lm], minlength=world)
        assert counts.max() - counts.min() <= 0.02 * len(lm) + 200, counts
