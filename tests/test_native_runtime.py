"""Native host runtime (csrc/runtime/host_runtime.cpp) against the numpy oracles,
plus a host-sanitizer (ASan + UBSan) build of its C++ self-test."""
import multiprocessing as mp
import os
import shutil
import subprocess

import numpy as np
import pytest
import torch

from apex_dqn_amd.envs.vector_envs import CartPoleVec
from apex_dqn_amd.replay.sumtree import SumTree, inverse_cdf_oracle
from apex_dqn_amd.runtime import native

pytestmark = pytest.mark.skipif(not native.available(), reason="native runtime not built")
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_sumtree_parity_with_numpy_oracle():
    rng = np.random.default_rng(0)
    cap = 3000
    a, b = SumTree(cap), native.NativeSumTree(cap)
    for _ in range(20):
        idx = rng.integers(0, cap, 400)
        idx[:50] = idx[50:100]                      # duplicates inside one call
        val = rng.random(400) * (rng.random(400) > 0.1)
        a.update(idx, val)
        b.update(idx, val)
        np.testing.assert_allclose(a.sum, b.sum, rtol=1e-12, atol=1e-9)
        np.testing.assert_array_equal(a.min, b.min)
    u = rng.random(1000) * a.total
    np.testing.assert_array_equal(b.find_prefix(u), inverse_cdf_oracle(b.sum[b.size2:b.size2 + cap], u))
    s = b.sample_stratified(256, np.random.default_rng(1))
    assert s.shape == (256,) and np.all(b.get(s) > 0)
    with pytest.raises(IndexError):
        b.update([cap], [1.0])


def test_cartpole_dynamics_match_numpy():
    E = 16
    ref, nat = CartPoleVec(E, seed=0), native.NativeCartPoleVec(E, seed=0)
    ref.reset()
    nat.reset()
    nat.state[:] = ref.state                        # same start state, then step both
    nat.t[:] = ref.t
    rng = np.random.default_rng(2)
    for _ in range(8):                              # short horizon: no terminations
        a = rng.integers(0, 2, E)
        o1, r1, d1, _ = ref.step(a)
        o2, r2, d2, _ = nat.step(a)
        assert not d1.any()
        np.testing.assert_allclose(o1, o2, rtol=1e-6, atol=1e-7)
        np.testing.assert_array_equal(d1, d2)
    # long run: episode bookkeeping and auto-reset
    lens = []
    for _ in range(3000):
        _, _, d, info = nat.step(rng.integers(0, 2, E))
        lens += list(info["episode_length"][d])
    assert lens and all(1 <= n <= 500 for n in lens)
    assert np.all(np.abs(nat.state) < 3.0)


def _reader(seq, payload, n_reads, q):
    lock = native.SeqLock(seq, payload)
    dst = torch.empty_like(payload)
    last, ok, torn = -1, 0, 0
    while ok < n_reads:
        v = lock.read_into(dst, last)
        if v >= 0:
            if not bool((dst == dst[0]).all()):
                torn += 1
            last, ok = v, ok + 1
    q.put(torn)


def test_seqlock_across_processes_never_tears():
    seq = torch.zeros(1, dtype=torch.int64).share_memory_()
    payload = torch.zeros(1 << 18, dtype=torch.float32).share_memory_()
    lock = native.SeqLock(seq, payload)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_reader, args=(seq, payload, 20, q))
    p.start()
    v = 0
    while p.is_alive() and v < 200000:
        v += 1
        lock.write(torch.full_like(payload, float(v)))
    p.join(timeout=120)
    assert q.get(timeout=10) == 0


@pytest.mark.skipif(shutil.which("g++") is None, reason="no host compiler")
def test_runtime_under_host_sanitizers(tmp_path):
    src = os.path.join(ROOT, "apex_dqn_amd", "csrc", "runtime")
    exe = str(tmp_path / "rt_selftest")
    cmd = ["g++", "-std=c++17", "-O1", "-g", "-fsanitize=address,undefined", "-fno-omit-frame-pointer",
           "-I", src, os.path.join(src, "tests", "runtime_selftest.cpp"), os.path.join(src, "host_runtime.cpp"),
           os.path.join(src, "nstep.cpp"), "-lpthread", "-o", exe]
    r = subprocess.run(cmd, capture_output=True, text=True)
    assert r.returncode == 0, r.stderr[-3000:]
    # verify_asan_link_order=0: tolerate other preloaded libraries in the environment
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:halt_on_error=1:verify_asan_link_order=0",
               UBSAN_OPTIONS="halt_on_error=1")
    r = subprocess.run([exe], capture_output=True, text=True, env=env, timeout=300)
    assert r.returncode == 0 and "OK" in r.stdout, (r.stdout + r.stderr)[-3000:]


@pytest.mark.parametrize("obs_shape,dtype", [((4,), np.int64), ((4,), np.float32)])
def test_native_nstep_builder_matches_numpy_oracle(obs_shape, dtype):
    """csrc/runtime/nstep.cpp == actors/nstep.py (the oracle): same transitions, in the
    same order, with the same keys / returns / discounts / initial priorities,
    across random episode ends and partial takes."""
    from apex_dqn_amd.actors.nstep import NStepBuilder
    from apex_dqn_amd.runtime import native
    if not native.available():
        pytest.skip("native runtime unavailable")
    E, A, n = 7, 5, 3
    ref = NStepBuilder(E, n, 0.97, obs_shape, dtype, env_id_offset=11)
    nat = native.NativeNStepBuilder(E, n, 0.97, obs_shape, dtype, env_id_offset=11)
    rng = np.random.default_rng(3)
    obs = rng.integers(0, 1000, (E,) + obs_shape).astype(dtype)
    got_r, got_n = [], []
    for t in range(200):
        q = rng.normal(size=(E, A)).astype(np.float32)
        a = rng.integers(0, A, E)
        r = rng.normal(size=E).astype(np.float32)
        d = rng.random(E) < 0.08
        nxt = rng.integers(0, 1000, (E,) + obs_shape).astype(dtype)
        ref.step(obs, q, a, r, d, nxt)
        nat.step(obs, q, a, r, d, nxt)
        assert ref.size == nat.size
        if t % 7 == 6:
            k = int(rng.integers(1, 40))
            for lst, b in ((got_r, ref), (got_n, nat)):
                out = b.get(k)
                if out is not None:
                    lst.append(out)
        obs = nxt
    for lst, b in ((got_r, ref), (got_n, nat)):
        out = b.get()
        if out is not None:
            lst.append(out)
    cat = lambda L, k: np.concatenate([o[k] for o in L])  # noqa: E731
    for k in ("S_t", "S_tpn", "A_t", "key", "env"):
        assert np.array_equal(cat(got_r, k), cat(got_n, k)), k
    for k in ("R", "Gamma", "priority"):
        np.testing.assert_allclose(cat(got_n, k), cat(got_r, k), rtol=1e-6, atol=1e-6)
    assert len(cat(got_r, "A_t")) > 500
