"""Batched NAVSIM evaluation producer.

The reference evaluates one token at a time: ``agent.compute_trajectory(agent_input)`` per token
inside ``run_pdm_score.py:72-102`` / ``run_create_submission_pickle.py:50-57`` (CPU feature build,
batch-1 forward). ``BatchedTrajectoryRunner`` produces the same ``{token: Trajectory}`` map with
the feature building and the forward batched on the GPU:

* agent inputs are loaded per token on the host (a token whose loader raises is reported failed
  and skipped, like the reference's per-token ``try/except``);
* features for a batch of up to ``batch_size`` scenes are built by the GPU feature builder in one
  call per sensor (``features.py``), the forward runs once per batch (numerics-checked);
* the DDIM start noise is drawn as ONE ``torch.randn(b, 20, 8, 2)`` per batch from the global
  generator, which yields exactly the values of ``b`` successive per-token ``torch.randn(1, 20, 8,
  2)`` draws of the reference (transfuser_model_v2.py:593; 320 = 20 x 16 normals per scene keeps
  PyTorch's 16-wide CPU normal fill aligned - tests/test_runner.py), so a seeded batched run equals a
  seeded per-token run scene for scene;
* ``run_distributed`` shards the token list over the ranks of a torch.distributed group (one
  process per GPU) and gathers the per-rank maps with one ``all_gather_object``;
* ``lanes`` > 1 keeps that many batches in flight on the GPU (model.py InFlightPlanner: the agent's
  handle plus clones, each a single-stream forward on a stream of its own); a batch is finished -
  synchronised, its lane's numerics flag read - before its lane takes the next one;
* failures are isolated per batch, as the reference isolates them per token (``run_pdm_score.py:77-100``:
  any exception marks the token invalid and the loop goes on): an exception while building a batch's
  features, launching its forward or finishing it marks that batch's tokens failed (``self.failed``)
  and the other batches - those already in flight on other lanes included - complete.

PDM scoring stays on the CPU (``pdm_score``, out of scope): feed it the returned trajectories.
"""
import collections
from typing import Callable, Dict, Iterable, List, Optional, Tuple

import numpy as np
import torch

from .agent import DiffusionDriveAgent, Trajectory
from .features import TransfuserFeatureBuilder


class BatchedTrajectoryRunner:
    def __init__(self, agent: DiffusionDriveAgent, batch_size: int = 64, device: Optional[int] = None,
                 lanes: int = 1):
        if batch_size < 1:
            raise ValueError("batch_size must be >= 1")
        if lanes < 1:
            raise ValueError("lanes must be >= 1")
        self.agent = agent
        self.batch_size = batch_size
        self.lanes = lanes
        self._clones: List = []
        self.device = agent._transfuser_model.device if device is None else device
        self.builder = TransfuserFeatureBuilder(agent._config, device=self.device)
        self.failed: List[Tuple[str, str]] = []

    def _features(self, inputs: List):
        """The batch's device features and its DDIM start noise (one draw per batch, in batch order)."""
        cfg = self.agent._config
        feats = self.builder.compute_features_batch(inputs)
        noise = torch.randn((len(inputs), cfg.num_modes, cfg.trajectory_sampling.num_poses, 2))
        return feats, noise

    def _finish(self, job) -> Dict[str, Trajectory]:
        """Wait for a launched batch; if its forward raised a numerics flag, re-run it directly in fp32."""
        tokens, feats, noise, out, model, stream = job
        if stream is not None:
            stream.synchronize()
        if model.numerics_flags(clear=True):
            with torch.no_grad():
                out = model.rerun_fp32(feats, noise)
        poses = out["trajectory"].cpu().numpy()
        return {t: Trajectory(np.ascontiguousarray(poses[i])) for i, t in enumerate(tokens)}

    def _planner(self):
        """(InFlightPlanner over the agent's handle + clones, each handle's stream count as found: the planner
        switches every lane to single-stream when there are several)."""
        from .model import InFlightPlanner
        model = self.agent._transfuser_model
        while len(self._clones) < self.lanes - 1:
            self._clones.append(model.clone())
        models = [model] + self._clones[:self.lanes - 1]
        saved = [m.stream_count() for m in models] if len(models) > 1 else []
        return InFlightPlanner(models=models), saved

    def close(self):
        """Release the lane clones' handles (the agent's own handle stays with the agent)."""
        for m in self._clones:
            m.close()
        self._clones = []

    def __del__(self):
        try:
            self.close()
        except Exception:  # noqa: BLE001 - interpreter shutdown
            pass

    def _fail(self, tokens: List[str], err: BaseException):
        self.failed.extend((t, repr(err)) for t in tokens)

    def _run_batches(self, batches: Iterable[Tuple[List[str], List]]) -> Dict[str, Trajectory]:
        """Software-pipelined: the next batch's host-side feature staging (the raw-sensor copy into the pinned
        stage) runs while up to ``lanes`` forwards are on the GPU; the oldest batch is finished (synchronised, its
        lane's numerics flag read - the feature kernels raise none) before its lane takes another batch, so every
        flag belongs to one forward. An exception in one batch's features, launch or finish fails that batch's
        tokens only."""
        # every lane runs single-stream while several are in flight; each handle's own count is restored after
        pl, saved = self._planner()
        for m in pl.lanes:
            m.numerics_flags(clear=True)
            if len(pl) > 1:
                m.set_streams(1)
        out: Dict[str, Trajectory] = {}
        pending = collections.deque()

        def finish_oldest():
            job = pending.popleft()
            try:
                out.update(self._finish(job))
            except Exception as e:  # noqa: BLE001 - per-batch isolation (run_pdm_score.py:77-100)
                self._fail(job[0], e)

        try:
            for tokens, inputs in batches:
                try:
                    feats, noise = self._features(inputs)
                except Exception as e:  # noqa: BLE001
                    self._fail(tokens, e)
                    continue
                # pending jobs sit on the lanes before next_index in round-robin order (the pointer advances only
                # after a successful launch), so when every lane is busy the oldest job is on the lane taken next:
                # its flags are read and cleared before another forward runs there
                if len(pending) == len(pl):
                    finish_oldest()
                lane = pl.lanes[pl.next_index]
                try:
                    with torch.no_grad(), pl.next_lane() as m:
                        s = torch.cuda.current_stream(m.device)  # the lane's stream (the caller's with one lane)
                        res = m.forward(feats, noise=noise, safe=False, stream=s)
                except Exception as e:  # noqa: BLE001
                    self._fail(tokens, e)
                    try:  # a partly issued forward may have raised flags: clear them before the lane's next batch
                        lane.numerics_flags(clear=True)
                    except Exception:  # noqa: BLE001 - the lane's next batch then fails on its own
                        pass
                    continue
                pending.append((tokens, feats, noise, res, m, s))
            while pending:
                finish_oldest()
        finally:
            for m, n in zip(pl.lanes, saved):
                m.set_streams(n)
        return out

    def run(self, tokens: Iterable[str], get_agent_input: Callable[[str], object]) -> Dict[str, Trajectory]:
        """{token: Trajectory} for every token whose input loads; failures land in ``self.failed``."""
        def batches():
            pend_t, pend_i = [], []
            for tok in tokens:
                try:
                    ai = get_agent_input(tok)
                except Exception as e:  # noqa: BLE001 - the reference marks the token invalid and goes on
                    self.failed.append((tok, repr(e)))
                    continue
                pend_t.append(tok)
                pend_i.append(ai)
                if len(pend_t) == self.batch_size:
                    yield pend_t, pend_i
                    pend_t, pend_i = [], []
            if pend_t:
                yield pend_t, pend_i

        return self._run_batches(batches())

    def run_distributed(self, tokens: List[str], get_agent_input: Callable[[str], object],
                        group=None) -> Dict[str, Trajectory]:
        """Shard ``tokens`` contiguously over the ranks, run locally, gather every rank's map."""
        import torch.distributed as dist
        world = dist.get_world_size(group) if dist.is_initialized() else 1
        rank = dist.get_rank(group) if dist.is_initialized() else 0
        per = (len(tokens) + world - 1) // world
        local = self.run(tokens[rank * per:(rank + 1) * per], get_agent_input)
        if world == 1:
            return local
        parts: List[Optional[dict]] = [None] * world
        dist.all_gather_object(parts, {t: tr.poses for t, tr in local.items()}, group=group)
        merged: Dict[str, Trajectory] = {}
        for p in parts:
            merged.update({t: Trajectory(np.asarray(v)) for t, v in p.items()})
        return merged
