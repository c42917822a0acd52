"""Overlapped actor / learner iterations for the training loop (config (e): BASELINE.json configs[4],
"7 self-play actor GPUs + 1 learner GPU").

The reference's loop is strictly sequential (MuZero_det_MADN/train_with_reward.py:244-292): play the
iteration's games with the current weights, save them, train, repeat -- so on N GPUs the learner idles while
the actors play and the actors idle through the learner's 2500 steps.  ``run_overlapped`` pipelines the two:

    prologue: actors play generation 0 (initial weights W_-1); it reaches the ring
    iteration i = 0 .. n-1:
        actors  play generation i+1 with the weights they hold        } concurrently
        learner trains iteration i on the ring (generations 0 .. i)   }
        deliver generation i+1 into the ring (every game exactly once)
        publish W_i to the actors (asynchronous; applied before they start generation i+2)

so generation g >= 1 is played with W_{g-2} where the sequential loop would use W_{g-1}: the policy is stale by
exactly ONE iteration, the price of an iteration time of max(self-play, learner) instead of their sum.  The
sequential order stays the default everywhere (``bench.py --workload train`` without ``--overlap``).

``run_overlapped`` only orders calls; the callables carry the transport:
  * one GPU (actor and learner in one process, ``concurrent=True``): generation i+1 is played in a worker
    thread on its own HIP stream while the learner's captured graph replays on another (ctypes releases the
    GIL inside the native self-play loop), delivery = ring.save_games_from_buffers, publish = push_to(net);
  * N ranks (actors 0..N-2, learner N-1): delivery = transfer.gather_packed (RCCL point-to-point) +
    ring.save_packed, publish = an ``async_op`` broadcast of the weight arena (transfer.broadcast_weights_async).
"""
from __future__ import annotations

import os
import threading


class _Done:
    def wait(self):
        return None


class OverlappedIterations:
    """The loop of ``run_overlapped`` as resumable steps (a benchmark times ``step()`` calls between its
    barriers).  Arguments as run_overlapped's."""

    def __init__(self, *, is_actor: bool, is_learner: bool, play, train, deliver, publish, concurrent: bool = False):
        self.is_actor, self.is_learner = bool(is_actor), bool(is_learner)
        self.play, self.train, self.deliver, self.publish = play, train, deliver, publish
        self.concurrent = bool(concurrent)
        if self.concurrent and self.is_actor and self.is_learner:
            # the DOG search beside a learner on the same GPU keeps 8 games per workgroup (188 workgroups at 1500
            # games, one per CU, 68 CUs left to the learner) instead of the standalone 6 (250): the overlapped DOG
            # iteration 11.98 -> 8.29 s (profiles/r5zk_dog_train.log).  (An explicit MUZ_DOG_GPW wins.)
            os.environ.setdefault("MUZ_DOG_GPW", "8")
        self.i = 0
        self.pending = _Done()

    def prologue(self):
        """Generation 0 (initial weights) into the ring."""
        self.deliver(0, self.play(0) if self.is_actor else None)

    def step(self):
        """Iteration i: generation i+1 played while iteration i trains; delivered; W_i published."""
        i = self.i
        self.pending.wait()                 # actors: W_{i-1} applied before generation i+1 starts
        games = None
        if self.concurrent and self.is_actor and self.is_learner:
            box, err = {}, []

            def actor():
                try:
                    box["g"] = self.play(i + 1)
                except BaseException as e:      # re-raised in the caller's thread
                    err.append(e)
            t = threading.Thread(target=actor, name=f"selfplay-gen{i + 1}")
            t.start()
            try:
                self.train(i)
            finally:
                t.join()
            if err:
                raise err[0]
            games = box["g"]
        else:
            if self.is_actor:
                games = self.play(i + 1)
            if self.is_learner:
                self.train(i)
        self.deliver(i + 1, games)
        self.pending = self.publish(i)
        self.i = i + 1

    def finish(self):
        self.pending.wait()
        self.pending = _Done()


def run_overlapped(iterations: int, *, is_actor: bool, is_learner: bool, play, train, deliver, publish,
                   concurrent: bool = False):
    """Run ``iterations`` overlapped iterations (module docstring).

    play(g) -> games of generation g (actors; None elsewhere) -- uses the weights the actor holds;
    train(i) -> None (learner);
    deliver(g, games) -> None: collective on every rank; the learner's ring receives generation g;
    publish(i) -> handle with .wait(): W_i from the learner to the actors (actors: the wait applies it);
    concurrent: play and train in two threads of this process (both roles on one GPU).
    Returns the number of generations delivered (iterations + 1)."""
    loop = OverlappedIterations(is_actor=is_actor, is_learner=is_learner, play=play, train=train, deliver=deliver,
                                publish=publish, concurrent=concurrent)
    loop.prologue()
    for _ in range(iterations):
        loop.step()
    loop.finish()
    return iterations + 1
