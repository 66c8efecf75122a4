"""csrc/raceline.hpp (the device raceline lookup of xref_mode RACELINE) compiled for the
host with AddressSanitizer and run against the oracle's ConstantSpeed loop
(planner.py:34-65, pinned by tests/golden/planner.npz): per-model mu below / inside /
above the friction profiles, NaN mu, starts across the lap including the mod-L wrap."""
import os
import shutil
import subprocess

import numpy as np
import pytest

from oracle import llampc_oracle as O

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")


@pytest.fixture(scope="module")
def harness(tmp_path_factory):
    if not os.path.exists(HIPCC) and not shutil.which("hipcc"):
        pytest.skip("hipcc not available")
    out = str(tmp_path_factory.mktemp("rl") / "raceline_host")
    cmd = [HIPCC, "-x", "hip", "--offload-arch=gfx950", "-O1", "-g", "-std=c++17",
           "-Xarch_host", "-fsanitize=address", "-Xarch_host", "-fno-omit-frame-pointer",
           f"-I{os.path.join(REPO, 'lla-mpc_amd', 'csrc')}", f"-I{os.path.join(REPO, 'include')}",
           os.path.join(REPO, "tests", "native", "raceline_host.cpp"), "-o", out]
    subprocess.run(cmd, check=True, capture_output=True)
    return out


@pytest.mark.parametrize("mode", ["global", "win"])
@pytest.mark.parametrize("name", ["ETHZ", "ETHZMobil"])
def test_raceline_walker_host_asan(harness, tmp_path, name, mode):
    """mode 'win': the speed profiles read through the launch's window (raceline.hpp
    SpeedWin, as the kernel prologue builds it) — the same references."""
    import sys
    sys.path.insert(0, os.path.join(REPO, "lla-mpc_amd"))
    from llampc.tracks import ETHZ, ETHZMobil
    tr = ETHZ('optimal', True) if name == "ETHZ" else ETHZMobil('optimal', True)
    knots, xy, speed, mus = tr.device_table()
    n, M = len(knots), len(mus)
    np.concatenate([[n, M], knots, xy.ravel(), speed.ravel(), mus]).astype(np.float64).tofile(tmp_path / "t.bin")
    H, Ts = 40, 0.02
    L = float(knots[-1])
    cases = []
    for mu in (0.2, mus[0], 0.5 * (mus[0] + mus[1]), mus[M // 2], mus[-1], 1.7, float("nan")):
        for s0, v0, scale in ((0.0, 1.0, 0.9), (0.37 * L, 2.5, 1.0), (L - 0.02, 3.0, 0.9), (L - 1e-9, 0.0, 0.9)):
            cases.append((mu, s0, v0, scale, Ts))
    np.concatenate([[H], np.ravel(cases)]).astype(np.float64).tofile(tmp_path / "c.bin")
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=0:abort_on_error=1")
    r = subprocess.run([harness, str(tmp_path / "t.bin"), str(tmp_path / "c.bin"), mode], capture_output=True,
                       text=True, env=env, check=True)
    got = np.array([list(map(float, ln.split())) for ln in r.stdout.strip().splitlines()]).reshape(len(cases), H, 2)
    td = np.load(os.path.join(REPO, "lla-mpc_amd", "llampc", "tracks", "data", "tracks.npz"))
    ref = O.RacelineRef(td[f"{name}_x"], td[f"{name}_y"], td[f"{name}_speeds"], td[f"{name}_mus"])
    for i, (mu, s0, v0, scale, _) in enumerate(cases):
        if np.isnan(mu):
            # the reference raises (bisect of a NaN arc length indexes past its spline
            # lists) from the second step on; the device walker propagates NaN instead
            xr, _ = O.constant_speed_from(s0, np.zeros(2), v0, ref, 1, Ts, scale, mu)
            np.testing.assert_allclose(got[i, 0], xr[:, 1], rtol=0, atol=1e-10)
            assert np.all(np.isnan(got[i, 1:]))
            continue
        xr, _ = O.constant_speed_from(s0, np.zeros(2), v0, ref, H, Ts, scale, mu)
        np.testing.assert_allclose(got[i], xr[:, 1:].T, rtol=0, atol=1e-10, err_msg=f"case {i} mu={mu} s0={s0}")
