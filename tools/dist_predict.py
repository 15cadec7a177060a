#!/usr/bin/env python3
"""Predicted step time of an N-way sharded solve WITH its collectives, from the per-rank device times
tools/dist_model.py measures on one MI355X (exchanges excluded there) and the exchange payloads ptzba_dist_info
reports for each rank.

Per LM trial a part-owned solve runs three all-reduces (sum) on the handle's stream, between kernels that depend
on them (so nothing overlaps them):
  X_SEP   the separator block, all N ranks                       sep_doubles x 8 B
  X_PART  the part's band inside a rank group (groups of > 1 rank) part_doubles x 8 B
  X_SCAL  the trial's scalars, all N ranks                         16 x 8 B (latency only)
Each collective is modelled as a ring all-reduce:  t = alpha + 2 (p - 1) / p * bytes / B
  B     = 153 GB/s, ONE xGMI link per direction (the single-ring bound; RCCL's channels over all 7
          links can only be faster for large messages -- the "links7" column divides the byte term by 7)
  alpha = 15 us per collective on 8 GPUs (an assumed RCCL small-message latency; no 8-GPU node was available to
          measure it: the prediction is only as good as this figure)
The step is the slowest rank's trial + its collectives; iterations/s follow at ~1 trial per iteration (config 3's
solves accept almost every trial).

  python tools/dist_predict.py profiles/r03dd_dist_model_c3.jsonl [profiles/r03dm_dist_model_c4.jsonl ...]
"""
import json
import sys

LINK_GBS = 153.0
ALPHA_US = 15.0


def t_allreduce_us(nbytes, p, links=1):
    if p <= 1 or nbytes <= 0:
        return 0.0
    return ALPHA_US + 2.0 * (p - 1) / p * nbytes / (LINK_GBS * links * 1e3)


def predict(recs):
    by_world = {}
    for r in recs:
        by_world.setdefault(r["world"], []).append(r)
    base = None
    out = []
    for world in sorted(by_world):
        rows = []
        for r in by_world[world]:
            x = r.get("exchange") or {}
            g = x.get("group_size", 1)
            terms = {}
            for links in (1, 7):
                if "exchanges" in x:  # round 4: every collective of the rank's trial, (kind, r0, group size, doubles)
                    t = sum(t_allreduce_us(8 * n, nr, links) for _, _, nr, n in x["exchanges"])
                else:
                    t = t_allreduce_us(8 * x.get("sep_doubles", 0), world, links) + \
                        t_allreduce_us(8 * x.get("part_doubles", 0), g, links) + \
                        t_allreduce_us(8 * x.get("scal_doubles", 0), world, links) + \
                        t_allreduce_us(8 * x.get("sys_doubles", 0), world, links)
                terms[links] = t / 1e3
            rows.append((r["wall_ms_per_trial"], terms, r))
        dev = max(t for t, _, _ in rows)
        step1 = max(t + e[1] for t, e, _ in rows)
        step7 = max(t + e[7] for t, e, _ in rows)
        fact = max(r["kernel_ms"].get("cholesky_solve", 0.0) for _, _, r in rows)
        if world == 1:
            base = dev
        out.append({"config": rows[0][2]["config"], "world": world, "rank_device_ms_per_trial": round(dev, 4),
                    "factorisation_ms": round(fact, 4),
                    "collectives_ms_1link": round(max(e[1] for _, e, _ in rows), 4),
                    "predicted_step_ms_1link": round(step1, 4), "predicted_step_ms_7links": round(step7, 4),
                    "predicted_speedup_1link": round(base / step1, 3) if base else None,
                    "predicted_speedup_7links": round(base / step7, 3) if base else None,
                    "model": f"ring all-reduce, alpha {ALPHA_US} us, {LINK_GBS} GB/s per xGMI link"})
    return out


def main():
    for path in sys.argv[1:]:
        recs = [json.loads(l) for l in open(path) if l.strip()]
        for row in predict(recs):
            print(json.dumps(row))


if __name__ == "__main__":
    main()
