import sys, numpy as np, torch
sys.path.insert(0, '.')
sys.path.insert(0, 'tests')
import test_gpu_brax as T
from oracle import oracle as O
name, kind = "brax_hover", O.ENV_BRAX_HOVER
n, L, seed = 256, 40, 3
env = T._env(n, name, L=L, seed=seed); env.reset()
rng = np.random.default_rng(seed)
e = O.BraxEnv(kind, episode_length=L)
for t in range(60):
    g = env.get_state()
    acts = rng.uniform(-1, 1, (n, 4)).astype(np.float32)
    obs, rew, te, tr, inf = env.step(torch.from_numpy(acts).cuda())
    tobs = inf["terminal_observation"].cpu().numpy(); obs = obs.cpu().numpy()
    for i in range(n):
        ep = int(g["episode"][i]) - 1
        e.reset_with(e.draw(seed, i, ep))
        e.s.qpos[:] = [float(x) for x in g["qpos"][i]]; e.s.qvel[:] = [float(x) for x in g["qvel"][i]]
        e.s.steps = int(g["step_count"][i])
        pre = np.concatenate([g["qpos"][i], g["qvel"][i]])
        r = e.step(acts[i])
        for nm, got, ref in (("obs", obs[i], r["obs"]), ("tobs", tobs[i], r["terminal_obs"])):
            d = np.abs(got.astype(np.float64) - ref)
            tol = 1e-5 * np.maximum(np.abs(ref), np.abs(pre)) + 1e-6
            if (d > tol).any():
                j = np.where(d > tol)[0]
                print(t, i, nm, j, got[j], ref[j], pre[j], acts[i], r["motor_commands"])
