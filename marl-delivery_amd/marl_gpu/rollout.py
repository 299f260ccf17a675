"""Device-resident MAPPO rollout glue.

Replaces the host side of ``MAPPOTrainer.collect_rollouts`` (MAPPO/trainer.py:154-290):
the per-agent ``.item()`` + LabelEncoder decode, the Python env loop, shaping, tracker,
per-agent featurization with H2D copies, and the GAE loop.  Here the policy's logits
are sampled on the device (``sample_actions``), the engine steps and featurizes straight
into the rollout buffers, and GAE runs as one kernel (``gae``).  Only the actor/critic
forward passes are the caller's (torch modules, as in the reference).
"""
from __future__ import annotations

import numpy as np
import torch

from ._lib import check, lib, ptr, stream_handle

ACTION_DIM = 15  # MAPPO/trainer.py:41


def sample_actions(logits: torch.Tensor, seed: int, offset: int, out=None):
    """``Categorical(logits=logits).sample()`` and ``.log_prob`` (MAPPO/trainer.py:141-143).

    logits: float32 [N, n_actions] on the device.  Returns (actions uint8 [N],
    log_probs float32 [N]).  The draw is the library's own Philox4x32-10 stream
    keyed by (seed, offset, row): deterministic, independent of launch shape.
    """
    if logits.dtype != torch.float32 or not logits.is_contiguous():
        logits = logits.float().contiguous()
    N, n_act = logits.shape
    if out is None:
        acts = torch.empty(N, dtype=torch.uint8, device=logits.device)
        lp = torch.empty(N, dtype=torch.float32, device=logits.device)
    else:
        acts, lp = out
    check(lib().mdl_sample_actions(ptr(logits), N, n_act, seed & (2**64 - 1), offset & (2**64 - 1), ptr(acts),
                                   ptr(lp), stream_handle(logits.device)), "mdl_sample_actions")
    return acts, lp


def sample_actions_dev(logits: torch.Tensor, seed: int, offset_dev: torch.Tensor, offset_add: int, out):
    """``sample_actions`` at offset ``offset_dev[0] + offset_add`` with the base read on the
    device (uint64 tensor [1]), so the launch can live in a replayed hipGraph."""
    if logits.dtype != torch.float32 or not logits.is_contiguous():
        logits = logits.float().contiguous()
    N, n_act = logits.shape
    acts, lp = out
    check(lib().mdl_sample_actions_dev(ptr(logits), N, n_act, seed & (2**64 - 1), ptr(offset_dev),
                                       offset_add & (2**64 - 1), ptr(acts), ptr(lp), stream_handle(logits.device)),
          "mdl_sample_actions_dev")
    return acts, lp


def gae(rewards, values, next_value, dones, gamma=0.99, gae_lambda=0.95, out=None):
    """Advantages and returns exactly as MAPPO/trainer.py:266-276 computes them.

    rewards, values: float32 [T, n]; dones: bool/uint8 [T, n]; next_value: float32 [n].
    ``GAMMA * GAE_LAMBDA`` is formed in double and rounded once, as the reference's
    Python expression does before it meets a float32 tensor.
    """
    T, n = rewards.shape
    dev = rewards.device
    r = rewards.float().contiguous()
    v = values.float().contiguous()
    nv = next_value.reshape(n).float().contiguous()
    d = dones.to(torch.uint8).contiguous()
    if out is None:
        adv = torch.empty((T, n), dtype=torch.float32, device=dev)
        ret = torch.empty((T, n), dtype=torch.float32, device=dev)
    else:
        adv, ret = out
    g = float(np.float32(gamma))
    gl = float(np.float32(gamma * gae_lambda))
    check(lib().mdl_gae(ptr(r), ptr(v), ptr(nv), ptr(d), T, n, g, gl, ptr(adv), ptr(ret), stream_handle(dev)),
          "mdl_gae")
    return adv, ret


class MappoRollout:
    """``collect_rollouts`` (MAPPO/trainer.py:154-290) on the device.

    env: a ``BatchedEnv`` built like the trainer's (tracker="mappo", shaping="mappo",
    max_other_robots=A-1, max_packages_obs=5, auto-reset on done).  actor(obs [E*A,6,H,W],
    vec [E*A,Dv]) -> logits [E*A, 15]; critic(gmap [E,4,H,W], gvec [E,Dg]) -> values [E]
    or [E, 1].  ``collect`` returns the reference's flattened batch.
    """

    def __init__(self, env, rollout_steps: int, seed: int = 0, gamma: float = 0.99, gae_lambda: float = 0.95):
        self.env = env
        self.T = int(rollout_steps)
        self.seed = int(seed)
        self.offset = 0
        self.gamma, self.gae_lambda = gamma, gae_lambda
        E, A = env.E, env.A
        if env._shape_run_end[0] < E:   # the buffers hold one [H, W]; a mixed-shape batch needs one rollout per group
            raise ValueError("MappoRollout: the engine's envs mix map shapes (build one engine per map shape)")
        H, W = env.grids[int(env.env_map[0])].shape
        dev = env.device
        f = dict(dtype=torch.float32, device=dev)
        T = self.T
        self.mb_obs = torch.zeros((T, E, A, 6, H, W), **f)
        self.mb_vector_obs = torch.zeros((T, E, A, env.actor_vec_dim), **f)
        self.mb_global_states = torch.zeros((T, E, 4, H, W), **f)
        self.mb_global_vector = torch.zeros((T, E, env.critic_vec_dim), **f)
        self.mb_actions = torch.zeros((T, E, A), dtype=torch.uint8, device=dev)
        self.mb_log_probs = torch.zeros((T, E, A), **f)
        self.mb_rewards = torch.zeros((T, E), **f)
        self.mb_dones = torch.zeros((T, E), dtype=torch.uint8, device=dev)
        self.mb_values = torch.zeros((T, E), **f)
        self.next_obs = env.obs_buffers(E, H, W)
        self._r_env = torch.zeros(E, dtype=torch.float64, device=dev)
        self._graph = None          # hipGraph of one whole rollout (collect(graph=True))
        self._graph_key = None      # (actor, critic, parameter addresses) the graph was captured with
        self._graph_out = None
        self._off_dev = torch.zeros(1, dtype=torch.int64, device=dev)   # sampler offset base (uint64 bits)

    def _slot(self, k):
        return dict(actor_map=self.mb_obs[k], actor_vec=self.mb_vector_obs[k], critic_map=self.mb_global_states[k],
                    critic_vec=self.mb_global_vector[k])

    @torch.no_grad()
    def collect(self, actor, critic, graph: bool = False):
        """One rollout of ``rollout_steps`` env steps.  graph=True: the first call runs
        eagerly and captures the whole rollout (policy forwards, sampling, steps,
        observations, GAE) as one hipGraph; later calls with the same actor/critic replay
        it -- bit-identical to eager calls (the sampler's offset base lives on the
        device and advances inside the graph).  The returned tensors are the graph's
        static buffers: consume them before the next collect."""
        if not graph:
            return self._run(actor, critic, False)
        # the graph reads the modules' parameters in place: replay only for the very same modules
        # (strong references, compared by identity) whose parameters still live at the captured
        # addresses (load_state_dict copies in place; rebinding ``param.data`` does not)
        ptrs = tuple(q.data_ptr() for m in (actor, critic) if hasattr(m, "parameters") for q in m.parameters())
        key = (actor, critic, ptrs)
        k0 = self._graph_key
        if self._graph is not None and k0[0] is actor and k0[1] is critic and k0[2] == ptrs:
            self._graph.replay()
            self.offset += self.T
            return self._graph_out
        out = self._run(actor, critic, False)        # this call's rollout, and the warm-up
        self._capture(actor, critic, key)
        return out

    def _capture(self, actor, critic, key):
        dev = self.env.device
        torch.cuda.synchronize(dev)
        self._off_dev.fill_(self.offset)
        s = torch.cuda.Stream(device=dev)
        s.wait_stream(torch.cuda.current_stream(dev))
        g = torch.cuda.CUDAGraph()
        off0 = self.offset
        with torch.cuda.stream(s):
            with torch.cuda.graph(g, stream=s):
                self._graph_out = self._run(actor, critic, True)
        torch.cuda.current_stream(dev).wait_stream(s)
        torch.cuda.synchronize(dev)
        self.offset = off0   # capture ran nothing
        self._graph, self._graph_key = g, key

    def _run(self, actor, critic, dev_offset: bool):
        env, T = self.env, self.T
        E, A = env.E, env.A
        env.build_obs(out=self._slot(0))              # current obs = f(current state, tracker)
        for step in range(T):
            obs = self.mb_obs[step]
            logits = actor(obs.reshape(E * A, *obs.shape[2:]), self.mb_vector_obs[step].reshape(E * A, -1))
            acts_lp = (self.mb_actions[step].view(-1), self.mb_log_probs[step].view(-1))
            if dev_offset:
                sample_actions_dev(logits, self.seed, self._off_dev, step, out=acts_lp)
            else:
                sample_actions(logits, self.seed, self.offset, out=acts_lp)
            self.offset += 1
            self.mb_values[step] = critic(self.mb_global_states[step], self.mb_global_vector[step]).reshape(E)
            # step + the next observations in one launch (MAPPO/trainer.py:229-286)
            env.step_obs(self.mb_actions[step], auto_reset=True,
                         out=(self._r_env, self.mb_rewards[step], self.mb_dones[step]),
                         obs_out=self._slot(step + 1) if step + 1 < T else self.next_obs)
        if dev_offset:
            check(lib().mdl_counter_add(ptr(self._off_dev), T, stream_handle(env.device)), "mdl_counter_add")
        next_value = critic(self.next_obs["critic_map"], self.next_obs["critic_vec"]).reshape(E)
        adv, ret = gae(self.mb_rewards, self.mb_values, next_value, self.mb_dones, self.gamma, self.gae_lambda)
        H, W = obs.shape[-2:]
        return (self.mb_obs.reshape(-1, 6, H, W), self.mb_vector_obs.reshape(T * E * A, -1),
                self.mb_global_states.reshape(T * E, 4, H, W), self.mb_global_vector.reshape(T * E, -1),
                self.mb_actions.reshape(-1).long(), self.mb_log_probs.reshape(-1),
                adv.reshape(T * E, 1).repeat(1, A).reshape(-1), ret.reshape(-1), self.mb_rewards)
