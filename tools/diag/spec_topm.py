"""Could the controller roll out its look-ahead models before the selection is known?  The
selection needs x_t (this tick's look-back error), but the window means change by one entry per
tick, so a superset of the next top-K could be known before x_t: per tick of the closed loop of
the device controller (restated by the oracle, ControllerOracle: the RK6 plant under the gradual
friction decay, the controller's own controls), whether the rolled-out set top-K_t + {argmin_t}
lies inside the M best models of a predictor known before x_t:
  prev      the previous tick's window means (its argsort)
  partial   the sum of the W - 1 window entries that stay (the one dropping out removed)
  partial+last  that sum plus the newest entry again (the coming error's estimate)
for M in a range; also the mean and max rank of the needed models under each predictor.  CPU
only (the oracle).  usage: python tools/diag/spec_topm.py [N] [ticks] [out.json]"""
import json
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [REPO, os.path.join(REPO, "lla-mpc_amd")]
from oracle import llampc_oracle as O  # noqa: E402

N = int(sys.argv[1]) if len(sys.argv) > 1 else 10000
T = int(sys.argv[2]) if len(sys.argv) > 2 else 200
OUT = sys.argv[3] if len(sys.argv) > 3 else None
MS = (11, 16, 24, 32, 48, 64, 96, 128)


def ranks_of(order, needed):
    pos = np.empty(order.size, dtype=np.int64)
    pos[order] = np.arange(order.size)
    return pos[needed]


def run(name, seed, x0, H=40, C=64, K=10, W=10):
    from llampc.mpc import generate_bank
    td = np.load(os.path.join(REPO, "lla-mpc_amd", "llampc", "tracks", "data", "tracks.npz"))
    ref = O.RacelineRef(td[f"{name}_x"], td[f"{name}_y"], td[f"{name}_speeds"], td[f"{name}_mus"])
    p = O.orca_params()
    shared = {k: p[k] for k in ("lf", "lr", "mass", "Iz", "Cm1", "Cm2", "Cr0", "Cr2")}
    orc = O.ControllerOracle(shared, generate_bank(N, seed=seed), ref, {"ETHZ": 656, "ETHZMobil": 440}[name],
                             H=H, C=C, K=K, W=W)
    plant = O.Vehicle.from_params(p)
    x = np.asarray(x0, dtype=np.float64)
    hits = {k: {m: 0 for m in MS} for k in ("prev", "partial", "partial+last")}
    maxrank = {k: [] for k in ("prev", "partial", "partial+last")}
    compared = 0
    for t in range(T):
        win = orc.win
        pre = None
        if win.count >= W:                        # predictors from the window BEFORE this tick's push
            prev_order = np.lexsort((np.arange(N), win.avg, np.isnan(win.avg)))
            part = win.win[:, 1:].sum(axis=1)     # the entries that stay after the roll
            part_order = np.lexsort((np.arange(N), part, np.isnan(part)))
            last = part + win.win[:, -1]          # ... plus the newest error again, as the next one's estimate
            last_order = np.lexsort((np.arange(N), last, np.isnan(last)))
            pre = {"prev": prev_order, "partial": part_order, "partial+last": last_order}
        o = orc.tick(x)
        if not o["warm"] and pre is not None:
            needed = np.unique(np.append(np.asarray(o["topk"], dtype=np.int64), int(o["best_model"])))
            compared += 1
            for k, order in pre.items():
                r = ranks_of(order, needed)
                maxrank[k].append(int(r.max()))
                for m in MS:
                    hits[k][m] += int(r.max() < m)
        plant.Df -= plant.Df / 2600.
        plant.Dr -= plant.Dr / 2600.
        xn, _ = O.sim_continuous(plant, x, o["u_seq"][:, 0].reshape(2, 1), [0, 0.02])
        x = xn[:, -1]
    return {"track": name, "N": N, "ticks": T, "compared": compared,
            "hit_rate": {k: {str(m): v / max(compared, 1) for m, v in d.items()} for k, d in hits.items()},
            "max_rank_of_needed": {k: {"mean": float(np.mean(v)) if v else None, "p99": float(np.percentile(v, 99)) if v else None,
                                       "max": int(max(v)) if v else None} for k, v in maxrank.items()}}


if __name__ == "__main__":
    d = np.load(os.path.join(REPO, "tests", "golden", "dyn_slice.npz"))
    td = np.load(os.path.join(REPO, "lla-mpc_amd", "llampc", "tracks", "data", "tracks.npz"))
    mob = td["ETHZMobil_init"]
    rows = [run("ETHZ", 0, d["states"][:, 0]), run("ETHZMobil", 1, [mob[0], mob[1], mob[2], 1.0, 0.0, 0.0])]
    for r in rows:
        print(json.dumps(r), flush=True)
    if OUT:
        json.dump(rows, open(OUT, "w"), indent=1)
