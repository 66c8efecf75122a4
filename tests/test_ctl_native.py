"""The controller tick's pure functions (csrc/ctl.hpp) compiled for the host with
AddressSanitizer and checked BITWISE against the NumPy restatement (oracle/llampc_oracle.py):
Philox4x32-10 against the Random123 known-answer vectors, the candidate sampler (noise, bound
clip, rate chains) against ``candidates_ctl``, the reference projection (projection.py:11-38,
track.py:147-160) against ``project_point`` on raceline windows of both tracks, and NumPy's
pairwise mean of the mu-hat ring (rt.py:339-341) against ``np.mean``."""
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
    out = str(tmp_path_factory.mktemp("ctl") / "ctl_host")
    cmd = [HIPCC, "-x", "hip", "--offload-arch=gfx950", "-O1", "-g", "-std=c++17",
           "-Xarch_host", "-fsanitize=address", "-Xarch_host", "-fno-omit-frame-pointer",
           f"-I{os.path.join(REPO, 'lla-mpc_amd', 'csrc')}", f"-I{os.path.join(REPO, 'include')}",
           os.path.join(REPO, "tests", "native", "ctl_host.cpp"), "-o", out]
    subprocess.run(cmd, check=True, capture_output=True)
    return out


def run(harness, tmp_path, mode, data):
    path = tmp_path / f"{mode}.bin"
    np.asarray(data, dtype=np.float64).tofile(path)
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=0:abort_on_error=1")
    r = subprocess.run([harness, mode, str(path)], capture_output=True, text=True, env=env, check=True)
    return r.stdout.strip().splitlines()


def test_philox_known_answers(harness, tmp_path):
    """Random123 kat_vectors for philox4x32_10, on the device code and on the oracle."""
    cases = [((0, 0, 0, 0), (0, 0), (0x6627e8d5, 0xe169c58d, 0xbc57ac4c, 0x9b00dbd8)),
             ((0xffffffff,) * 4, (0xffffffff,) * 2, (0x408f276d, 0x41c83b0e, 0xa20bc7c6, 0x6d5451fd)),
             ((0x243f6a88, 0x85a308d3, 0x13198a2e, 0x03707344), (0xa4093822, 0x299f31d0),
              (0xd16cfe09, 0x94fdcceb, 0x5001e420, 0x24126ea1))]
    out = run(harness, tmp_path, "philox", [v for c, k, _ in cases for v in (*c, *k)])
    for (c, k, want), line in zip(cases, out):
        assert tuple(map(int, line.split())) == want
        assert tuple(int(x) for x in O.philox4x32_10(np.array([c], dtype=np.uint32), k)[0]) == want


@pytest.mark.parametrize("C,H,has_prev,tick,seed", [(8, 20, False, 0, 2), (64, 40, True, 17, 2), (5, 7, True, 2**33 + 5, 2**40 + 9)])
def test_candidates_bitwise(harness, tmp_path, C, H, has_prev, tick, seed):
    rng = np.random.RandomState(C + H)
    uprev = np.array([0.3, -0.05])
    sigma = (0.05, 0.02)
    umin, umax, rate = (-0.1, -0.35), (1.0, 0.35), (None, 5.0)
    prev = np.column_stack([rng.uniform(-0.2, 1.1, H), rng.uniform(-0.4, 0.4, H)]) if has_prev else None
    ns = [O.SQRT3 * sigma[0], O.SQRT3 * sigma[1]]
    data = [C, H, int(has_prev), tick, seed, *uprev, *ns, *umin, *umax, -1.0, 5.0 * 0.02]
    if has_prev:
        data += list(prev.ravel())
    got = np.array(list(map(float, run(harness, tmp_path, "cands", data)))).reshape(C, H, 2)
    want = O.candidates_ctl(C, H, prev, uprev, sigma, umin, umax, rate, 0.02, tick, seed)
    np.testing.assert_array_equal(got, want)
    # the sampler's own properties: bounds, steering rate, candidate 0 = the base
    assert np.all(got >= np.array(umin)) and np.all(got <= np.array(umax))
    d = np.diff(np.concatenate([np.broadcast_to(uprev, (C, 1, 2)), got], axis=1)[:, :, 1], axis=1)
    assert np.all(np.abs(d) <= 0.1 + 1e-15)


@pytest.mark.parametrize("name", ["ETHZ", "ETHZMobil"])
def test_projection_bitwise(harness, tmp_path, name):
    """ref_project_dist = projection.py:11-38 per segment; the index = np.argmin (first
    minimum) of project_fast on raceline[:, p:p+10], including the short windows at the end."""
    td = np.load(os.path.join(REPO, "lla-mpc_amd", "llampc", "tracks", "data", "tracks.npz"))
    rl = np.array([td[f"{name}_x"], td[f"{name}_y"]], dtype=np.float64)
    n = rl.shape[1]
    rng = np.random.RandomState(7)
    cases = []
    for p0 in list(rng.randint(0, n - 10, 40)) + [0, n - 10, n - 5, n - 2]:
        base = rl[:, p0 + rng.randint(0, min(9, n - 1 - p0))]
        for _ in range(3):
            cases.append((*(base + rng.normal(0, 0.05, 2)), p0))
        cases.append((*rl[:, min(p0 + 3, n - 1)], p0))           # exactly on a vertex
    out = run(harness, tmp_path, "project", [n, *rl.ravel(), *np.ravel(cases)])
    ref = O.RacelineRef(td[f"{name}_x"], td[f"{name}_y"], td[f"{name}_speeds"], td[f"{name}_mus"])
    for (px, py, p0), line in zip(cases, out):
        vals = line.split()
        seg = ref.raceline[:, int(p0):int(p0) + 10]
        d = np.array([O.project_point((px, py), seg[:, i], seg[:, i + 1])[1] for i in range(seg.shape[1] - 1)])
        _, j = ref.project_fast(px, py, seg)
        assert int(vals[0]) == j
        np.testing.assert_array_equal(np.array(list(map(float, vals[1:]))), d)


def test_pairwise_ring_mean(harness, tmp_path):
    """np.mean(np.array(hist)[-S:]) and np.mean(top-K values) (rt.py:339-341) through the
    device's ring: NumPy's pairwise order, bitwise."""
    rng = np.random.RandomState(3)
    data, want = [], []
    for n, cap in ((1, 20), (5, 20), (8, 20), (10, 32), (13, 20), (20, 20), (17, 64), (64, 64)):
        v = rng.randn(cap) * rng.exponential(1, cap)
        first = int(rng.randint(0, cap))
        seq = np.array([v[(first + i) % cap] for i in range(n)])
        data += [n, cap, first, *v]
        want.append(np.mean(seq))
    got = np.array(list(map(float, run(harness, tmp_path, "mean", data))))
    np.testing.assert_array_equal(got, np.array(want))
