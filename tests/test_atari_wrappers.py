"""DQN Atari wrapper stack (frame-skip + max-pool, no-op starts, episodic life,
reward clipping) on the deterministic FakeALE emulator -- the reference has none
of these (``env.py:3-4`` is a bare ``gym.make``)."""
import numpy as np

from apex_dqn_amd.envs.vector_envs import AtariPreprocess, AtariWrapperVec, FakeALE, make_vec_env


def _env(n=2, **kw):
    return AtariWrapperVec([FakeALE(seed=i) for i in range(n)], **kw)


def test_frame_skip_sums_and_clips_rewards():
    env = _env(1, noop_max=0, clip_rewards=False, episodic_life=False)
    env.reset()
    emu = env.envs[0]
    t0 = emu.t
    _, r, _, _ = env.step([0])
    assert emu.t == t0 + 4                        # 4 emulator frames per agent step
    expect = sum(5.0 for t in range(t0 + 1, t0 + 5) if t % 7 == 0)
    assert r[0] == expect
    env2 = _env(1, noop_max=0, clip_rewards=True, episodic_life=False)
    env2.reset()
    rs = [env2.step([0])[1][0] for _ in range(10)]
    assert set(rs) <= {0.0, 1.0} and 1.0 in rs    # clipped to sign(r)


def test_max_pool_over_last_two_frames():
    emu = FakeALE(seed=0)
    env = AtariWrapperVec([emu], noop_max=0, episodic_life=False)
    env.reset()
    # replay the same 4 frames on a twin emulator to build the expected pooled frame
    twin = FakeALE(seed=0)
    twin.reset_game()
    frames = []
    for _ in range(4):
        twin.act(env.actions[0])
        frames.append(twin.getScreenRGB())
    obs, _, _, _ = env.step([0])
    expect = AtariPreprocess()(np.maximum(frames[2], frames[3]))
    np.testing.assert_array_equal(obs[0], expect)


def test_noop_starts_are_bounded_and_random():
    starts = []
    for s in range(12):
        env = AtariWrapperVec([FakeALE(seed=0)], noop_max=30, seed=s)
        env.reset()
        starts.append(env.envs[0].t)
    assert all(0 <= t <= 30 for t in starts) and len(set(starts)) > 3


def test_episodic_life_and_real_game_over():
    env = _env(1, noop_max=0, episodic_life=True, clip_rewards=False)
    env.reset()
    emu = env.envs[0]
    dones, real, rets = [], [], []
    for _ in range(60):
        _, _, d, info = env.step([0])
        dones.append(bool(d[0]))
        real.append(bool(info["real_done"][0]))
        if info["real_done"][0]:
            rets.append(info["episode_return"][0])
            assert emu.lives() == 3                    # emulator reset right after game over
            break
    # 3 lives x 60 frames = 180 frames = 45 agent steps: 2 life losses, then game over
    assert sum(dones) >= 3 and sum(real) == 1
    first_life = dones.index(True)
    assert first_life == 14 and not real[first_life]   # frame 60 falls in step 15
    assert rets and rets[0] > 0                        # unclipped game return reported once


def test_factory_fake_ale_shapes():
    env = make_vec_env("fake_ale", "PongNoFrameskip-v4", 3, 6, seed=1)
    obs = env.reset()
    assert obs.shape == (3, 84, 84) and obs.dtype == np.uint8 and env.action_dim == 6
    obs, r, d, info = env.step(np.zeros(3, np.int64))
    assert obs.shape == (3, 84, 84) and r.shape == (3,) and d.shape == (3,)


def test_envs_write_frames_into_a_given_buffer():
    """``step(actions, out=buf)`` (the actor's zero-copy path into the replay's pinned
    staging buffer, actors/gpu_actor.py _env_step) returns ``buf`` holding exactly the
    frames a plain step returns, for the synthetic env and the ALE wrapper stack."""
    from apex_dqn_amd.envs.vector_envs import make_vec_env
    for backend in ("synthetic", "fake_ale"):
        a, b = (make_vec_env(backend, "PongNoFrameskip-v4", 6, 6, seed=3) for _ in range(2))
        assert a.frame_out and b.frame_out
        np.testing.assert_array_equal(a.reset(), b.reset())
        rng = np.random.default_rng(0)
        for _ in range(40):
            act = rng.integers(0, 6, 6)
            buf = np.full((6, 84, 84), 7, np.uint8)
            fa, ra, da, _ = a.step(act)
            fb, rb, db, _ = b.step(act, out=buf)
            assert fb is buf
            np.testing.assert_array_equal(fa, fb)
            np.testing.assert_array_equal(ra, rb)
            np.testing.assert_array_equal(da, db)
