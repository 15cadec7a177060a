#!/usr/bin/env python3
"""What splitting each shared phase's factorisation over its rank group would buy (round-4 VERDICT item 4), predicted
from the measured per-rank device times (tools/dist_model.py records) and the library's own rank plans (host-only
ptzba_dist_plan_export / ptzba_dist_rank_phases on the BASELINE problem's coupling window).

Today every member of a phase group -- a shared leaf (X_PART), an inner separator (X_SUB), the root
separator (X_SEP) -- factors that phase's columns redundantly after the group's exchange.  The split alternative is a
1-D block-cyclic distribution of the phase's tile columns over its g ranks in blocks of 4 columns, with one panel
broadcast per block (delayed updates: make_plan's DT = 4).  Per shared phase of L levels (~L tile columns):

  unsplit   L * t_avg                          t_avg = the rank's measured cholesky_solve / its level count
  split     max(L * t_chain, L * t_avg / g)  + ceil(L / 4) * t_bcast
            t_chain = 7.5 us: a chain-bound level (config 3, rocprof r05z: 26 levels x 7.44 us; sweep 3.7 us + launch,
                      tile round trip, panel GEMMs) -- a split cannot make a level shorter than its pivot chain
            t_bcast = alpha + 2 (g - 1) / g * bytes / B  (ring, as tools/dist_predict.py), bytes = 4 x 32 columns x
                      (half the phase's rows + every later phase's rows) x 8 B
The rank's step becomes  wall - fact + fact_split + its current collectives (dist_predict's).  Output: one JSON line
per (config, world) with the current and the split prediction at 1 and 7 xGMI links.

  python tools/dist_split_model.py c3_n1.jsonl+profiles/r04i_dist_model_c3.jsonl profiles/r04i_dist_model_c4.jsonl
  (c3_n1.jsonl = the first line of profiles/r04g_dist_model_c3.jsonl: config 3's N = 1 row, as dist_predict used it)
"""
import json
import math
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "pan-tilt-zoom-slam_amd"), os.path.join(ROOT, "tools")]

import dist_predict  # noqa: E402

T_CHAIN_US = 7.5


def t_bcast_us(nbytes, g, links):
    return dist_predict.t_allreduce_us(nbytes, g, links)


def split_fact_ms(rec, phases, win_rows, links):
    """phases: [(lv0, lv1, kind, r0, nr)] of the rank (dist_plan_export); win_rows[q]: rows of phase q."""
    fact = rec["kernel_ms"]["cholesky_solve"]
    levels = max(1, rec["solver"]["levels"])
    t_avg = fact * 1e3 / levels  # us per level
    out = fact * 1e3
    nbc = 0
    for q, (lv0, lv1, kind, r0, nr) in enumerate(phases):
        if nr < 2:
            continue
        L = lv1 - lv0
        later_rows = sum(win_rows[q + 1:])
        nbytes = 4 * 32 * (win_rows[q] / 2 + later_rows) * 8
        nb = math.ceil(L / 4)
        nbc += nb
        split = max(L * T_CHAIN_US, L * t_avg / nr) + nb * t_bcast_us(nbytes, nr, links)
        out += split - L * t_avg
    return out / 1e3, nbc


def main():
    import ptzba
    import synthetic
    for arg in sys.argv[1:]:  # "a.jsonl+b.jsonl": one config's records from several runs (e.g. its N = 1 row)
        recs = [json.loads(l) for path in arg.split("+") for l in open(path) if l.strip()]
        cfg = recs[0]["config"]
        prob = synthetic.make_problem(cfg, seed=0)
        win = ptzba.frame_coupling_window(prob.n_pose, prob.frame, prob.landmark)
        del prob
        cur = {(r["world"]): r for r in dist_predict.predict(recs)}
        base = cur[1]["rank_device_ms_per_trial"]
        by_world = {}
        for r in recs:
            by_world.setdefault(r["world"], []).append(r)
        for world in sorted(by_world):
            row = {"config": cfg, "world": world, "current_speedup_1link": cur[world]["predicted_speedup_1link"],
                   "current_speedup_7links": cur[world]["predicted_speedup_7links"]}
            if world > 1:
                for links in (1, 7):
                    steps, facts, nbcs = [], [], []
                    for r in by_world[world]:
                        ph = ptzba.dist_plan_export(win, world, r["rank"])[4]
                        rows = [3 * (e - s) for (_, _, _, s, e) in ptzba.dist_rank_phases(win, world, r["rank"])]
                        fs, nbc = split_fact_ms(r, ph, rows, links)
                        x = r.get("exchange") or {}
                        coll = sum(dist_predict.t_allreduce_us(8 * n, nr, links) for _, _, nr, n in
                                   x.get("exchanges", [])) / 1e3
                        steps.append(r["wall_ms_per_trial"] - r["kernel_ms"]["cholesky_solve"] + fs + coll)
                        facts.append(fs)
                        nbcs.append(nbc)
                    row[f"split_step_ms_{links}link"] = round(max(steps), 4)
                    row[f"split_speedup_{links}link"] = round(base / max(steps), 3)
                    row[f"split_factorisation_ms_{links}link"] = round(max(facts), 4)
                row["panel_broadcasts_per_trial"] = max(nbcs)
                row["chain_floor_ms"] = round(max(r["solver"]["levels"] for r in by_world[world]) * T_CHAIN_US / 1e3, 4)
            row["model"] = (f"split: max(L*{T_CHAIN_US} us, L*t_avg/g) + ceil(L/4) panel broadcasts, ring alpha "
                            f"{dist_predict.ALPHA_US} us, {dist_predict.LINK_GBS} GB/s per link")
            print(json.dumps(row), flush=True)


if __name__ == "__main__":
    main()
