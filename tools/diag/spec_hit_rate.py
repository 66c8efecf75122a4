"""Would the controller tick gain from speculating on the previous tick's selection (verdict r04
#4b)?  The closed loop of the device controller, restated by the oracle (ControllerOracle: the
RK6 plant under the gradual friction decay, the controller's own controls), counts per tick
whether the K + 1 look-ahead models (the top-K and the selected model) equal the previous
tick's as a multiset — a tick whose rollouts could all start before the selection arrives —
and, separately, whether the selected model alone stayed.  CPU only (the oracle).
usage: python tools/diag/spec_hit_rate.py [N] [ticks] [out.json]"""
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
    prev = prev_sel = None
    full = all_hits = sel_hits = 0
    for t in range(T):
        o = orc.tick(x)
        if not o["warm"]:
            cur = sorted([int(i) for i in o["topk"]] + [int(o["best_model"])])
            if prev is not None:
                full += 1
                all_hits += cur == prev
                sel_hits += int(o["best_model"]) == prev_sel
            prev, prev_sel = cur, int(o["best_model"])
        plant.Df -= plant.Df / 2600.
        plant.Dr -= plant.Dr / 2600.
        xn, _ = O.sim_continuous(plant, x, o["u_seq"][:, 0].reshape(2, 1), [0, 0.02])
        x = xn[:, -1]
    return {"track": name, "N": N, "ticks": T, "compared": full, "all_slots_same": all_hits,
            "all_slots_rate": all_hits / max(full, 1), "selected_same": sel_hits, "selected_rate": sel_hits / max(full, 1)}


if __name__ == "__main__":
    d = np.load(os.path.join(REPO, "tests", "golden", "dyn_slice.npz"))
    td = np.load(os.path.join(REPO, "lla-mpc_amd", "llampc", "tracks", "data", "tracks.npz"))
    mob = td["ETHZMobil_init"]
    rows = [run("ETHZ", 0, d["states"][:, 0]), run("ETHZMobil", 1, [mob[0], mob[1], mob[2], 1.0, 0.0, 0.0])]
    for r in rows:
        print(json.dumps(r), flush=True)
    if OUT:
        json.dump(rows, open(OUT, "w"), indent=1)
