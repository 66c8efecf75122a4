"""Tick inputs of the BASELINE configs: synthetic-but-physical states from the
RK6 plant (Dynamic.sim_continuous, dynamic.py:59-74) under the config's friction change
(rt.py:125-141), the ConstantSpeed reference (planner.py:12-67) and candidate sequences.

  config 2 (ETHZ, gradual):   states from DYN states[:, 470] driven by the recorded ETHZ
                              controls, D <- D (1 - 1/2600) per tick, starting 100 ticks into
                              the decay (rt.py:125-130)
  config 3 (ETHZMobil, sudden): no stored Mobil trajectory exists, so the car
                              starts at the track's (x_init, y_init, psi_init) with vx ~ U[0.5, 3],
                              vy ~ U[-0.3, 0.3], omega ~ U[-4, 4]; controls pwm ~ U[-0.1, 1] and
                              delta a random walk in [-0.35, 0.35], |d delta| <= 0.1 (seed 3);
                              nine ticks of D -= D/22 (rt.py:132-141)

One tick's pack is [x_prev 6 | u_prev 2 | x_now 6 | uprev 2 | xref 2(H+1) | U 2CH] (float64),
the layout of ShardedBank.make_plan_in.  The plant runs on the device (the library's RK6)."""
from __future__ import annotations

import numpy as np


def default_scenario(track_name: str) -> str:
    return "sudden" if track_name == "ETHZMobil" else "gradual"


def mobil_controls(T: int, seed: int = 3) -> tuple[np.ndarray, np.ndarray]:
    """Config 3's synthetic start state offsets and controls: (x0 tail [vx, vy, omega], u [2, T])."""
    rng = np.random.RandomState(seed)
    v0 = np.array([rng.uniform(0.5, 3.0), rng.uniform(-0.3, 0.3), rng.uniform(-4.0, 4.0)])
    u = np.empty((2, T))
    d = 0.0
    for t in range(T):
        u[0, t] = rng.uniform(-0.1, 1.0)
        d = float(np.clip(d + rng.uniform(-0.1, 0.1), -0.35, 0.35))
        u[1, t] = d
    return v0, u


def scenario_ticks(track_name: str, H: int, C: int, T: int, scenario: str | None = None, device: int = 0,
                   cand_seed: int = 2, dyn_path: str | None = None) -> np.ndarray:
    """T tick packs [T, 16 + 2(H+1) + 2CH] of the config's scenario (see the module text)."""
    from llampc.models import Dynamic
    from llampc.mpc.controller import CandidateGenerator
    from llampc.mpc.planner import ConstantSpeed
    from llampc.params import ORCA
    from llampc.tracks import ETHZ, ETHZMobil, dyn_slice
    p = ORCA()
    plant = Dynamic(**p, device=device)
    track = ETHZ('optimal', True) if track_name == "ETHZ" else ETHZMobil('optimal', True)
    scenario = scenario or default_scenario(track_name)
    gen = CandidateGenerator(C, H, seed=cand_seed)
    Ts = 0.02
    if track_name == "ETHZMobil":
        v0, u_rec = mobil_controls(T + 1)
        x = np.array([track.x_init, track.y_init, track.psi_init, *v0])
    else:
        d = np.load(dyn_path) if dyn_path else dyn_slice()
        u_rec = d["inputs"]
        x = d["states"][:, 0].copy()
    if scenario == "gradual":
        k0 = 100                                # ticks into the decay
        Df, Dr = p["Df"] * (1 - 1 / 2600.) ** k0, p["Dr"] * (1 - 1 / 2600.) ** k0
    else:
        Df, Dr = p["Df"], p["Dr"]
    packs, projidx = [], 0
    for t in range(T + 1):
        u = u_rec[:, t % u_rec.shape[1]]
        plant.Df, plant.Dr = Df, Dr
        xn, _ = plant.sim_continuous(x, u.reshape(2, 1), [0, Ts])
        x_next = xn[:, -1]
        if t >= 1:
            mu = (Df + Dr) / (9.81 * p["mass"])
            xref, projidx, _ = ConstantSpeed(x_next[:2], x_next[3], track, H, Ts, projidx, curr_mu=mu, scale=0.9)
            if projidx > track.lap_projidx:     # rt.py:287-296
                projidx = 0
            U = gen(None, u)
            packs.append(np.concatenate([x, u, x_next, u, xref.ravel(), U.ravel()]))
        x = x_next
        if scenario == "gradual":
            Df -= Df / 2600.
            Dr -= Dr / 2600.
        elif 2 <= t < 11:                       # nine ticks of D -= D/22 (rt.py:132-140)
            Df -= Df / 22.
            Dr -= Dr / 22.
    return np.stack(packs[:T])


def unpack(pk: np.ndarray, H: int, C: int) -> dict:
    """A pack's fields: x_prev, u_prev, x_now, uprev, xref [2, H+1], U [C, H, 2]."""
    return dict(x_prev=pk[0:6], u_prev=pk[6:8], x_now=pk[8:14], uprev=pk[14:16],
                xref=pk[16:16 + 2 * (H + 1)].reshape(2, H + 1), U=pk[16 + 2 * (H + 1):].reshape(C, H, 2))
