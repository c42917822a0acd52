#!/usr/bin/env python3
"""Self-play throughput benchmark: det-MADN, B = 4096 games per GPU, 50-simulation Gumbel MuZero.

Metric (BASELINE.json): self-play env-steps/s (+ MCTS sims/s), det-MADN batch 4096, 1/2/4/8 GPU.
  * one bench "step" = 32 x 4096 complete games per rank with a 50-simulation search per move (SURVEY
    §8d b), played 4096 at a time: the self-play batch is 4096 concurrent games, and a game that ends
    hands its lane to the next game (muz_detmadn_selfplay_stream).  --games 0 times the reference's
    own unit instead, one play_n_games_v3 call of 4096 games whose batch shrinks as games finish;
  * env-steps = sum of recorded turns (idx) over all games and ranks, exactly game_agent.py:140;
  * sims/s = searches x S / time.
Weak scaling: every rank plays its own 4096 games (games are independent; no data-path collective).
Timing: W untimed warm-up steps, then K steps between barrier + synchronize on both sides,
max over ranks.  Rank 0 prints ONE JSON line.

Weights are seeded random (Flax-default init; no checkpoints are available), data is synthetic
(self-generated games), arithmetic is fp32 end to end (the north star's 1e-5 fp32 target).
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

BATCH = 4096
# One det bench step streams 32 x 4096 games through the 4096 concurrently played games (lanes): a lane
# whose game ends starts the next game, so searches run on a full batch instead of shrinking with the
# finished games as one play_n_games_v3 batch does (its tail averages ~54 % active games).  Each game's
# record is identical to the batch call's (tests/test_gpu_selfplay.py::test_stream_equals_batch).  Only
# the drain at the end of a step (the last games of the queue finishing) runs on a partial batch: ~12 %
# of a step with 8 generations, ~6 % with 16, ~3 % with 32 (a continuously running actor has none).
# Records of 131072 games (T = 500) take ~75 GB of the GPU's 288 GB HBM.
STREAM_GENERATIONS = 32
S = 50
D = 25
MAX_STEPS = 500
TEMP = 1.0
PLAYERS = 2
# Algorithmic work per simulation: DynamicsNetwork4 529,280 MAC + PredictionNetwork4 404,544 MAC
# (recomputed in DESIGN.md) -> FLOP = 2 x MAC.
FLOP_PER_SIM = 2 * (529_280 + 404_544)
# What the kernel executes per simulation: the FiLM sub-graph (Dense_0 -> Dense_1|Dense_2) depends on the
# action only and is tabulated once per weight set (muz_net_prepare), and one-hot products are row
# gathers: Dyn4 491,904 MAC (d3, d4, 2 ResBlocks, d5, Dense_6|7 latent rows, heads) + Pred4 404,544 MAC.
EXEC_FLOP_PER_SIM = 2 * (491_904 + 404_544)
PEAK_FP32_MFMA_TFLOPS = 157.3   # MI355X_MICROARCH.md: Peak FP32 (matrix), dense
PEAK_HBM_GBS = 8000.0           # MI355X_MICROARCH.md: HBM3E
# Config (e) learner step (train_with_reward.py:24-164): per sample Repr2 once (3,380,480 MAC at C = 34),
# Pred4 K + 1 = 11 times (404,544), Dyn4 K = 10 times (529,280) -> 13,123,264 MAC forward; x2 FLOP, x3 for
# forward + backward, x batch 128
LEARNER_FLOP_PER_STEP = 3 * 2 * 13_123_264 * 128
# MuZero_DOG/train.py's learner step on the DOG slice's nets: Repr 3,380,480 + 11 x Pred4 at A = 806 (504,640) + 10 x
# Dyn4 at A = 806 (679,424, its one-hot layers counted as the reference computes them) = 15,725,760 MAC per sample
DOG_LEARNER_FLOP_PER_STEP = 3 * 2 * 15_725_760 * 128
# Config (c): classic MADN 4p teams.  Algorithmic MAC per simulation (one branch evaluated):
# decision = StochasticDynamics afterstate path + Pred4(A=4); chance = StochasticDynamics chance path + Pred4.
CLASSIC_PLAYERS = 4
# Algorithmic MAC per simulation of the stochastic search: each simulation expands ONE node -- a decision
# node's child (action dynamics 518,432 + PredictionNetwork4(A=4) on the afterstate 401,984 = 920,416) or a
# chance node's child (chance dynamics 491,904 + 401,984 = 893,888); paths alternate decision / chance
# levels, so the mean of the two, 907,152, is used (JAX evaluates both branches: 1,814,304).
CLASSIC_FLOP_PER_SIM = 2 * 907_152
# Config (d): DOG 2v2, 1024 games per GPU (8192 over 8 GPUs), uniform random legal policy.
DOG_BATCH = 1024
DOG_TURNS_PER_LAUNCH = 1024     # one muz_dog_random_play launch plays 1024 turns of every game (~10 ms)
DOG_LAUNCHES_PER_STEP = 32      # one bench step = 32 launches (~0.3 s: the default 3 steps time ~1 s)

# DOG MuZero slice (--workload dog --policy muzero): MuZero_DOG/train.py:337-338 (S = 100, D = 50), 1500 games per GPU
# (train.py:332 num_games_per_iteration; the random-policy config (d) is 1024).
DOG_MZ_GAMES = 1500
# FLOP per simulation at A = 806, counted as the reference would compute it (one-hot Dense layers as matmuls, like
# the det count): DynamicsNetwork4 679,424 MAC (Dense_0 806 x 64 and the one-hot rows of Dense_6 / 7, 806 x 128, are
# the A-dependent parts) + PredictionNetwork4 504,640 MAC (policy logits 128 x 806).  Executed on the device:
# 996,544 MAC (one-hot rows are gathers; the action-only FiLM sub-graph is a per-action table).
DOG_MZ_SIMS, DOG_MZ_DEPTH, DOG_MZ_TURNS_PER_STEP = 100, 50, 8
DOG_MZ_FLOP_PER_SIM = 2 * (679_424 + 504_640)
DOG_MZ_EXEC_FLOP_PER_SIM = 2 * 996_544


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--batch", type=int, default=None,
                    help=f"games per GPU (default: {BATCH}; dog: {DOG_BATCH}, dog --policy muzero: {DOG_MZ_GAMES})")
    ap.add_argument("--sims", type=int, default=None, help="MCTS simulations (det / classic 50, dog muzero 100)")
    ap.add_argument("--depth", type=int, default=None, help="MCTS max depth (det / classic 25, dog muzero 50)")
    ap.add_argument("--max-steps", type=int, default=MAX_STEPS)
    ap.add_argument("--cpu-seconds", type=float, default=20.0, help="budget of the CPU-baseline sample (1 core + all cores)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--games", type=int, default=-1,
                    help="det: games per step streamed through the --batch lanes (default 32 x batch; 0 = one "
                         "batch of --batch games, the reference's play_n_games_v3 call)")
    ap.add_argument("--train-steps", type=int, default=2500, help="train workload: learner steps per iteration")
    ap.add_argument("--overlap", action="store_true",
                    help="train workload: actors play iteration i+1 while the learner trains iteration i "
                         "(pipeline.run_overlapped; weights one iteration staler than the reference's loop)")
    ap.add_argument("--workload", choices=("det", "classic", "dog", "train", "env", "selftest"), default="det",
                    help="det = the BASELINE.json headline (config b); classic = config (c); dog = config (d)")
    ap.add_argument("--env-variant", type=int, choices=(0, 1, 2, 3, 4, 5), default=0,
                    help="env workload: 0 = kernel by batch size, 1 = one game per lane, 2 = one game per 32 lanes")
    ap.add_argument("--records", action="store_true",
                    help="dog: record every turn (muz_dog_random_play_record), pack the records each step and gather "
                         "them to rank 0 (RCCL point-to-point at N > 1) inside the timed region -- config (d) as "
                         "BASELINE.json names it")
    ap.add_argument("--game", choices=("det", "dog"), default="det",
                    help="train workload: det = train_with_reward.py (det-MADN 4p), dog = MuZero_DOG/train.py (the DOG "
                         "slice's nets, A = 806, DogSelfPlay records) -- BASELINE configs[4]'s 'full MuZero_DOG train "
                         "loop'")
    ap.add_argument("--policy", choices=("random", "muzero"), default="random",
                    help="dog: the reference's config (d) random legal policy, or the DOG MuZero slice (repr net with "
                         "its LayerNorm head + Dyn4 / Pred4 at A = 806 + Gumbel search, MuZero_DOG/train.py's S = 100, "
                         "D = 50)")
    ap.add_argument("--split", action="store_true",
                    help="strong scaling (SURVEY §8e): --batch is the WHOLE job's batch, split evenly over the ranks "
                         "(det 4096 -> 2048/1024/512 per GPU); default is weak scaling, --batch games per GPU")
    args = ap.parse_args()
    dog_mz = args.workload == "dog" and args.policy == "muzero"
    if args.batch is None:
        args.batch = (DOG_MZ_GAMES if dog_mz else DOG_BATCH) if args.workload == "dog" else BATCH
    if args.sims is None:
        args.sims = DOG_MZ_SIMS if dog_mz else S
    if args.depth is None:
        args.depth = DOG_MZ_DEPTH if dog_mz else D
    args.job_batch = args.batch
    if args.split:
        world = int(os.environ.get("WORLD_SIZE", str(args.gpus)))
        if args.batch % world:
            raise SystemExit(f"--split: batch {args.batch} is not divisible by {world} ranks")
        args.batch //= world
    if args.games < 0:
        args.games = STREAM_GENERATIONS * args.batch
    return args


def launch_ranks(n):
    """`bench.py --gpus N` without a launcher around it: start N fresh child processes of this script, one per
    GPU, with RANK / LOCAL_RANK / WORLD_SIZE / MASTER_ADDR / MASTER_PORT set (what torch.distributed.run
    would set), wait for all of them and exit with the worst status.  This parent never touches the GPU; each
    child initialises its own device and the process group.  Rank 0 prints the job's JSON line."""
    import socket
    import subprocess
    backend = os.environ.get("MUZ_BENCH_BACKEND", "nccl")
    if backend == "nccl":
        import torch   # device_count() does not initialise the GPU on this image
        have = torch.cuda.device_count()
        if n > have:
            raise SystemExit(f"bench.py --gpus {n}: only {have} GPU(s) visible")
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:], env=env))
    # poll every child: the first one that fails ends the job (the others would wait forever in the
    # process-group rendezvous or an RCCL collective), and MUZ_BENCH_TIMEOUT (seconds) bounds the whole job
    import time
    limit = float(os.environ.get("MUZ_BENCH_TIMEOUT", "0") or 0)
    t0, code = time.monotonic(), 0
    while True:
        codes = [p.poll() for p in procs]
        bad = [c for c in codes if c not in (None, 0)]
        if bad or all(c == 0 for c in codes):
            code = bad[0] if bad else 0
            break
        if limit and time.monotonic() - t0 > limit:
            print(f"bench.py: ranks still running after {limit:.0f} s, terminating", file=sys.stderr)
            code = 124
            break
        time.sleep(0.2)
    for p in procs:
        if p.poll() is None:
            p.terminate()
    for p in procs:
        try:
            p.wait(timeout=30)
        except subprocess.TimeoutExpired:
            p.kill()
            p.wait()
    return code


def dist_env():
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    return rank, world, local


def cpu_cores():
    """Host cores for the all-core CPU baseline: the process's affinity set, capped by OMP_NUM_THREADS when
    the environment sets it (the GPU box grants a 16-CPU share of a larger machine and sets it to 16)."""
    aff = len(os.sched_getaffinity(0))
    omp = os.environ.get("OMP_NUM_THREADS")
    return (min(aff, int(omp)) if omp and omp.isdigit() else aff), aff


def cpu_baseline(seconds, sims, depth, max_steps, lanes=16):
    """SURVEY §8(d)'s CPU timing: the C++ restatement of the reference algorithm (oracle/cpu_selfplay.cpp:
    det-MADN env + Repr2/Dyn4/Pred4 fp32 + Gumbel MuZero, OpenMP over game lanes; checked against the NumPy
    oracle by tests/test_cpu_baseline.py) plays streamed 2p games on the host for `seconds` at 1 thread and
    again at all cores.  The reference's own JAX-CPU path cannot run here (no jax in the image)."""
    from oracle import cpu_selfplay as CS
    from oracle import detmadn as dm
    from oracle import nets as ON
    C = dm.num_channels(PLAYERS)
    net = CS.CpuNet(ON.init_params(C, seed=0), C)
    cores, aff = cpu_cores()
    half = seconds / 2
    one = net.bench(PLAYERS, dm.SELFPLAY_RULES, lanes, sims, depth, max_steps, TEMP, 0, 1, half)
    allc = net.bench(PLAYERS, dm.SELFPLAY_RULES, lanes, sims, depth, max_steps, TEMP, 0, cores, half)
    v1 = one["env_steps"] / one["elapsed"]
    vn = allc["env_steps"] / allc["elapsed"]
    return {"value": round(vn, 2), "unit": "env_steps/s", "cores": cores, "kind": "port",
            "value_1core": round(v1, 2), "value_allcores": round(vn, 2), "cores_affinity": aff,
            "sims_per_s_allcores": round(allc["searches"] * sims / allc["elapsed"], 1),
            "sample": f"C++ restatement of the reference algorithm (oracle/cpu_selfplay.cpp, fp32 AVX2/FMA, OpenMP): "
                      f"det-MADN {PLAYERS}p streamed self-play, {lanes} game lanes per thread, S={sims} D={depth}, "
                      f"{half:.0f} s at 1 thread ({one['env_steps']} env-steps) and {half:.0f} s at {cores} threads "
                      f"({allc['env_steps']} env-steps); affinity shows {aff} CPUs"}


# The committed measurement summaries the bench lines quote, named explicitly (not picked by filename order): each is
# re-taken on the round's kernel by profiles/r5i_measure.sh and checked for the kernel it describes.
MEASURED = {
    "traffic": "profiles/r5i_traffic.json",           # HBM bytes per k_gumbel_search launch (FETCH_SIZE x2 + WRITE_SIZE)
    "pmc": "profiles/r5i_pmc.json",                   # TCP_TCC_READ_REQ, SQ_VALU_MFMA_BUSY_CYCLES, ... (k_gumbel_search)
    "loop": "profiles/r5i_loop_bench.log",            # the weight-stream MFMA loop alone (profiles/loop_bench.hip)
    "dog_traffic": "profiles/r6b_dog_traffic.json",   # HBM bytes per k_dog_search launch (FETCH_SIZE x2 + WRITE_SIZE), 6 games / WG
    "classic_traffic": "profiles/r6b_classic_traffic.json",   # the same for k_stochastic_search (config c)
    "dog_kernel_stats": "profiles/r6ae_dog_kernel_stats.csv",  # rocprofv3 --kernel-trace --stats of the DOG MuZero line
}


def measured_kernel_avg_ms(key, kernel):
    """The average duration (ms) of `kernel` in a committed rocprofv3 kernel-stats CSV of the same bench command:
    (ms, source) or (None, None)."""
    import csv
    path = os.path.join(ROOT, MEASURED[key])
    if not os.path.exists(path):
        return None, None
    with open(path) as f:
        for r in csv.DictReader(f):
            if kernel in r.get("Name", ""):
                return float(r["AverageNs"]) / 1e6, MEASURED[key]
    return None, None


def _measured_json(key, kernel):
    path = os.path.join(ROOT, MEASURED[key])
    if not os.path.exists(path):
        return None, None
    t = json.load(open(path))
    if t.get("kernel") != kernel:
        return None, None
    return t, MEASURED[key]


def measured_traffic(key="traffic", kernel="k_gumbel_search"):
    """HBM bytes per launch of `kernel` from its committed PMC summary (profiles/summarize_profile.py from
    rocprofv3 FETCH_SIZE / WRITE_SIZE passes of this bench): (bytes, source) or (None, None)."""
    t, src = _measured_json(key, kernel)
    return (t.get("bytes_per_launch"), src) if t else (None, None)


L2_SERVED_TBS = 18.8   # MI355X_MICROARCH.md, rows shared by every workgroup, served by the XCD's L2 (16.8-18.8)


def measured_l2_reads():
    """L1 -> L2 read bytes per k_gumbel_search launch (TCP_TCC_READ_REQ_sum, 128-byte requests) and the MFMA-busy
    fraction (SQ_VALU_MFMA_BUSY_CYCLES) from the round's PMC summary: (bytes, mfma_busy_frac, source)."""
    t, src = _measured_json("pmc", "k_gumbel_search")
    if not t:
        return None, None, None
    per = t.get("per_launch_mean", {})
    l2 = per["TCP_TCC_READ_REQ_sum"] * 128 if "TCP_TCC_READ_REQ_sum" in per else None
    return l2, t.get("mfma_busy_frac"), src


def measured_loop_ceiling():
    """The search kernel's weight-stream MFMA loop alone (profiles/loop_bench.hip: 14 resident 256x256 fp32
    layers on a 16-row LDS tile, a barrier per layer, every CU busy) from the round's loop-bench log: its TFLOP/s /
    the fp32 MFMA peak is the fraction the kernel could reach if its serial phases (tree walk, LayerNorm passes,
    epilogues, heads, backup) cost nothing.  Returns a dict or None."""
    import re
    path = os.path.join(ROOT, MEASURED["loop"])
    if not os.path.exists(path):
        return None
    for line in open(path):
        m = re.match(r"grid 256 lb_base: .*MFMA busy ([0-9.]+) of SIMD cycles, clock ([0-9.]+) GHz, ([0-9.]+) TFLOP/s",
                     line)
        if m:
            busy, clk, tf = (float(x) for x in m.groups())
            return {"frac": round(tf / PEAK_FP32_MFMA_TFLOPS, 4), "tflops": tf, "mfma_busy": busy, "clock_GHz": clk,
                    "source": MEASURED["loop"]}
    return None


def setup(args):
    rank, world, local = dist_env()
    if world != args.gpus:
        raise SystemExit(f"bench.py --gpus {args.gpus} but WORLD_SIZE={world}")
    import torch
    import muzpkg
    muzpkg.load()
    dist = None
    backend = os.environ.get("MUZ_BENCH_BACKEND", "nccl")
    if backend == "gloo":      # CPU rehearsal of the launcher / reduction path (tests/test_bench_launcher.py)
        device = torch.device("cpu")
    elif backend == "gloo_gpu":   # N ranks sharing the visible GPU(s), gloo collectives: a one-GPU rehearsal of the
        device = torch.device("cuda", local % torch.cuda.device_count())   # N-rank job (launch, barriers, reductions)
        torch.cuda.set_device(device)
    else:
        device = torch.device("cuda", local)
        torch.cuda.set_device(device)
    if world > 1:
        import torch.distributed as tdist
        tdist.init_process_group("gloo" if backend == "gloo_gpu" else backend, init_method="env://")
        dist = tdist
    return rank, world, dist, device


def parallelism(args, world):
    if args.split:
        return f"dp{world} strong: {args.job_batch} games split {args.batch}/GPU"
    return f"dp{world} weak: {args.batch} games/GPU, independent games"


def synchronize(device):
    import torch
    if device.type == "cuda":
        torch.cuda.synchronize(device)


def beat(msg):
    """Progress line on stderr (long steps would otherwise look hung to a watchdog)."""
    print(f"[bench {time.strftime('%H:%M:%S')}] {msg}", file=sys.stderr, flush=True)


def timed_region(dist, fn, steps):
    """barrier + synchronize, K steps, synchronize + barrier; returns the rank's elapsed seconds."""
    import torch
    dev = torch.device("cuda") if torch.cuda.is_available() else torch.device("cpu")
    if dist is not None:
        dist.barrier()
    synchronize(dev)
    t0 = time.perf_counter()
    for k in range(steps):
        fn(k)
        beat(f"step {k + 1}/{steps} issued")
    synchronize(dev)
    if dist is not None:
        dist.barrier()
    return time.perf_counter() - t0


def sum_max(dist, device, sums, elapsed):
    """Sum work over ranks, max of wall time (the slowest rank bounds the job)."""
    import torch
    if dist is None:
        return sums, elapsed
    if dist.get_backend() == "gloo":
        device = torch.device("cpu")
    t = torch.tensor([float(x) for x in sums], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.SUM)
    m = torch.tensor([elapsed], dtype=torch.float64, device=device)
    dist.all_reduce(m, op=dist.ReduceOp.MAX)
    return [x.item() for x in t], m[0].item()


def dog_cpu_baseline(seconds, lanes=8):
    """SURVEY §8(d)'s CPU timing for config (d): the C++ restatement of the DOG env (oracle/cpu_dog.cpp: dog.py's
    806-action legality, transitions and deals with the engine's counter-RNG deal keys and random legal action,
    finished games restarted; checked against the NumPy oracle by tests/test_cpu_baseline_dog.py) on the host for
    `seconds`, at 1 thread and at all cores."""
    from oracle import cpu_selfplay as CS
    from oracle import dog as dg
    cores, aff = cpu_cores()
    half = seconds / 2
    one = CS.dog_bench(4, dg.SELFPLAY_RULES, lanes, 5, 1, half)
    allc = CS.dog_bench(4, dg.SELFPLAY_RULES, lanes, 5, cores, half)
    v1 = one["env_steps"] / one["elapsed"]
    vn = allc["env_steps"] / allc["elapsed"]
    return {"value": round(vn, 2), "unit": "env_steps/s", "cores": cores, "kind": "port",
            "value_1core": round(v1, 2), "value_allcores": round(vn, 2), "cores_affinity": aff,
            "sample": f"C++ restatement of the reference DOG env (oracle/cpu_dog.cpp, OpenMP): 4p teams uniform random "
                      f"legal play, {lanes} games per thread restarted when finished, {half:.0f} s at 1 thread "
                      f"({one['env_steps']} env-steps, {one['games']} games finished) and {half:.0f} s at {cores} "
                      f"threads ({allc['env_steps']} env-steps); affinity shows {aff} CPUs"}


# k_dog_play's per-turn critical path, measured with the stamp build (profiles/diag_dog_stamps.py,
# profiles/r4c_dog_stamps_wave.log: 256-thread workgroup, wave priority on, round 4's wave-parallel env_step):
# thread 0 of each game's workgroup, shader-clock ticks per game-turn by phase (relative shares; the stamps
# themselves add ~10 %).  Round 3 (lane-0 env_step, profiles/r4c_dog_stamps_lane0.log): 4628 ticks of 15317.
DOG_PHASES = {"reset check / restart": 447, "base checks + barrier": 7072, "mask words + choice": 1788,
              "env_step (wave 0)": 3383, "barrier": 120, "deal": 1495}
# the phases a fully parallel turn keeps: the 448-thread base checks and their barrier, the one-wave action
# choice, the turn-end barrier and the (already wave-parallel) deal; wave 0's env_step (its lookups and board
# updates are still one dependent chain) and the reset check are the serial remainder a faster kernel would remove
DOG_IRREDUCIBLE = ("base checks + barrier", "mask words + choice", "barrier", "deal")


def dog_latency_model(avg_ms, games, turns, launch_bytes):
    """Config (d)'s roofline is a latency bound, not a bandwidth fraction: each game is one workgroup whose
    turn is a serial chain (checks -> barrier -> choice -> one-lane env_step -> barrier -> deal); all games
    are resident at once (4 workgroups of 7 waves per CU), so a launch takes about one chain per turn.
    `achieved` = measured us per game-turn; `peak` = the lower bound of that chain once lane 0's env_step
    and the reset check are fully parallelised (the irreducible phases' share of the stamp-build turn applied
    to the measured turn); frac = peak / achieved (time-like: 1.0 = nothing left to parallelise).  HBM
    traffic is negligible (bytes_per_launch / launch time)."""
    tot = sum(DOG_PHASES.values())
    us_per_turn = avg_ms * 1e3 / turns
    share = sum(DOG_PHASES[k] for k in DOG_IRREDUCIBLE) / tot
    floor_us = us_per_turn * share
    return {"bound": "latency", "kernel": "k_dog_play", "unit": "us/game-turn", "achieved": round(us_per_turn, 3),
            "peak": round(floor_us, 3), "frac": round(share, 4),
            "ceiling": "per-turn chain without its serial part: " + " + ".join(DOG_IRREDUCIBLE),
            "phase_share": {k: round(v / tot, 4) for k, v in DOG_PHASES.items()},
            "phase_ticks_per_turn_stamp_build": DOG_PHASES, "games_resident": games, "avg_launch_ms": round(avg_ms, 5),
            "hbm_gbs": round(launch_bytes / (avg_ms * 1e-3) / 1e9, 2), "traffic": None,
            "note": "per-phase shares from the stamp build (profiles/r4c_dog_stamps_wave.log); r4: env_step on all "
                    "64 lanes of wave 0 (ballot / readlane lookups, 4628 -> 3383 ticks; 6.18 -> 5.80 us/turn, "
                    "profiles/r4c_dog_bench_*.json); r3: 4-wave workgroups (no register spills; 6.81 -> 6.17 us/turn) "
                    "and the turn's serial part at raised wave priority, profiles/r3_dog_prio_ab.log"}


def dog_muzero_cpu_baseline(seconds, sims, depth, lanes=4, temperature=1.0, seed=5):
    """SURVEY §8(d)'s CPU timing for the DOG MuZero line: the C++ restatement of the slice (oracle/cpu_dog.cpp: the
    34-channel encoding, the DOG RepresentationNetwork + Dyn4 / Pred4 at A = 806 in fp32 AVX2/FMA, mctx's Gumbel
    search with lane-order sums (oracle/cpu_search.hpp), dog.py transitions with the engine's deal keys, finished
    games restarted; checked against the NumPy oracle -- networks at 1e-5, the search bit for bit, the self-play turn
    action for action -- by tests/test_cpu_baseline_dog.py) plays `lanes` games per thread on the host for `seconds`,
    at 1 thread and at all cores.  Same parameter init as the device line (init seed 2)."""
    from oracle import cpu_selfplay as CS
    from oracle import dog as dg
    from oracle import dog_muzero as DM
    net = CS.CpuNet(DM.init_params(seed=2), DM.NUM_CHANNELS)
    cores, aff = cpu_cores()
    half = seconds / 2
    one = net.dog_bench(dg.SELFPLAY_RULES, lanes, sims, depth, temperature, seed, 1, half)
    allc = net.dog_bench(dg.SELFPLAY_RULES, lanes, sims, depth, temperature, seed, cores, half)
    v1 = one["env_steps"] / one["elapsed"]
    vn = allc["env_steps"] / allc["elapsed"]
    return {"value": round(vn, 2), "unit": "env_steps/s", "cores": cores, "kind": "port",
            "value_1core": round(v1, 2), "value_allcores": round(vn, 2), "cores_affinity": aff,
            "sims_per_s_allcores": round(allc["searches"] * sims / allc["elapsed"], 1),
            "sample": f"C++ restatement of the DOG MuZero slice (oracle/cpu_dog.cpp + oracle/cpu_search.hpp, fp32 "
                      f"AVX2/FMA, OpenMP): 4p teams, {lanes} games per thread, S={sims} D={depth}, {half:.0f} s at 1 "
                      f"thread ({one['env_steps']} env-steps, {one['searches']} searches) and {half:.0f} s at {cores} "
                      f"threads ({allc['env_steps']} env-steps, {allc['searches']} searches); affinity shows {aff} CPUs"}


def run_dog_muzero(args):
    """Config (d) with the DOG MuZero slice: B 4-player DOG games per GPU played by the MuZero policy
    (game_agent_dog.DogSelfPlay: legal mask -> encode -> RepresentationNetwork + Pred4 -> Gumbel search at A = 806
    with Dyn4 / Pred4 -> step, finished games restarting in place).  One bench step = DOG_MZ_TURNS_PER_STEP turns of
    every game; env-steps = games x turns.  Roofline: k_dog_search's algorithmic FLOP over its HIP-event time."""
    import numpy as np
    import torch
    rank, world, dist, device = setup(args)
    from exploring_muzero_on_dog_amd import game_agent_dog as GA
    from exploring_muzero_on_dog_amd import muzero_dog as MD
    net = MD.DeviceDogNet(MD.init_muzero_params(2), device=device)
    sp = GA.DogSelfPlay(net, args.batch, args.sims, args.depth, 1.0, seed=4 + 1000 * rank, device=device)
    K = DOG_MZ_TURNS_PER_STEP
    ev = []
    from exploring_muzero_on_dog_amd import lib as L
    clib = L.load()
    orig = clib.muz_dog_gumbel_search

    # HIP events on the launching stream around every search launch: the C call alone, so the host's argument
    # preparation in muzero_dog.gumbel_muzero_policy stays outside (profiles/r4zf_dog_kernel_stats.csv)
    def timed_search(*a):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        rc = orig(*a)
        e1.record()
        ev.append((e0, e1))
        return rc

    def step(k):
        sp.play(K)

    sp.play(1)                           # warmup turn (workspace, first launches)
    for _ in range(args.warmup):
        step(-1)
    games0 = int(sp.episodes.sum().item())     # games finished before the timed region
    clib.muz_dog_gumbel_search = timed_search
    try:
        elapsed = timed_region(dist, step, args.steps)
    finally:
        clib.muz_dog_gumbel_search = orig
    search_ms = sum(a.elapsed_time(b) for a, b in ev)
    turns = args.steps * K
    (steps_done, sms, games), elapsed = sum_max(dist, device, [args.batch * turns, search_ms,
                                                             int(sp.episodes.sum().item()) - games0], elapsed)
    if rank != 0:
        if dist is not None:
            dist.destroy_process_group()
        return
    avg_ms = sms / (turns * world)
    # frac counts the FLOP the search executes: one-hot rows as gathers, the action-only FiLM
    # sub-graph as a table; the reference-form count (one-hot Dense layers as matmuls) is reported beside it
    achieved = args.batch * args.sims * DOG_MZ_EXEC_FLOP_PER_SIM / (avg_ms * 1e-3) / 1e12
    achieved_alg = args.batch * args.sims * DOG_MZ_FLOP_PER_SIM / (avg_ms * 1e-3) / 1e12
    traffic, traffic_src = measured_traffic("dog_traffic", "k_dog_search")
    # the same kernel's average by rocprofv3 on this command (frac on both timing bases)
    prof_ms, prof_src = measured_kernel_avg_ms("dog_kernel_stats", "k_dog_search")
    # k_dog_search's games per workgroup as the library launches it (was hard-coded)
    gpw = int(clib.muz_dog_search_games_per_workgroup(args.batch))
    out = {
        "metric": "self-play env steps/sec + MCTS sims/sec, DOG 2v2 MuZero policy (config d, DOG MuZero slice)",
        "value": round(steps_done / elapsed, 2), "unit": "env_steps/s", "n_gpus": world, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": round(1000 * elapsed / args.steps, 4), "higher_is_better": True,
        "scaling": "strong" if args.split else "weak", "vs_baseline": None, "dtype": "f32",
        "data": "synthetic (seeded deals, seeded random fp32 weights, counter-RNG Gumbel noise)",
        "sims_per_s": round(steps_done * args.sims / elapsed, 1), "games_finished": int(games),
        "config": {"workload": f"DOG 4p teams, {args.batch} games/GPU, MuZero policy (DOG RepresentationNetwork + "
                               f"Dyn4 / Pred4 at A = 806), Gumbel search S={args.sims} D={args.depth}, {K} turns of "
                               f"every game per step, finished games restart in place", "games_per_gpu": args.batch,
                   "num_simulations": args.sims, "max_depth": args.depth, "turns_per_step": K,
                   "parallelism": parallelism(args, world)},
        "roofline": {"bound": "mfma", "kernel": "k_dog_search", "achieved": round(achieved, 3), "peak": PEAK_FP32_MFMA_TFLOPS,
                     "unit": "TFLOP/s", "frac": round(achieved / PEAK_FP32_MFMA_TFLOPS, 4), "avg_launch_ms": round(avg_ms, 4),
                     "flop_per_sim": DOG_MZ_EXEC_FLOP_PER_SIM, "flop_counted": "executed (one-hot rows as gathers)",
                     "reference_form_flop_per_sim": DOG_MZ_FLOP_PER_SIM,
                     "reference_form_frac": round(achieved_alg / PEAK_FP32_MFMA_TFLOPS, 4),
                     "frac_rocprof": None if prof_ms is None else round(
                         args.batch * args.sims * DOG_MZ_EXEC_FLOP_PER_SIM / (prof_ms * 1e-3) / 1e12 /
                         PEAK_FP32_MFMA_TFLOPS, 4),
                     "rocprof_avg_launch_ms": None if prof_ms is None else round(prof_ms, 4),
                     "rocprof_source": prof_src,
                     "workgroups": -(-args.batch // gpw), "games_per_workgroup": gpw,
                     "traffic": None if traffic is None else round(traffic),
                     "traffic_achieved_tbs": None if traffic is None else round(traffic / (avg_ms * 1e-3) / 1e12, 3),
                     "traffic_source": traffic_src,
                     "note": f"{gpw} games per 16-row workgroup ({'two per wave' if gpw == 16 else 'one per wave'}): "
                             f"{args.batch} games occupy {-(-args.batch // gpw)} of the 256 CUs; a workgroup's "
                             f"search time is its serial chain of 100 simulations"},
    }
    if world == 1 and not args.no_cpu_baseline:
        out["cpu_baseline"] = dog_muzero_cpu_baseline(args.cpu_seconds, args.sims, args.depth)
    print(json.dumps(out), flush=True)
    if dist is not None:
        dist.destroy_process_group()


def run_dog(args):
    """Config (d): B DOG games per GPU (4p teams, MuZero_DOG/game_agent.py:12-23 rules) advanced by the
    uniform random legal policy; one bench step = one batched turn (muz_dog_random_turn: legal mask, action
    choice, env_step / no_step and any deal in one launch).  env-steps = turns of games not yet finished."""
    import torch
    rank, world, dist, device = setup(args)
    from exploring_muzero_on_dog_amd import dog as DG
    T, L = DOG_TURNS_PER_LAUNCH, DOG_LAUNCHES_PER_STEP
    rp = DG.RandomPlay(args.batch, seed=4 + 1000 * rank, fused=True)
    warm = torch.zeros(args.batch, dtype=torch.int32, device=device)
    env_steps = torch.zeros(args.batch, dtype=torch.int32, device=device)
    episodes = torch.zeros(args.batch, dtype=torch.int32, device=device)
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(args.steps)]
    traj = DG.DogTrajectory(args.batch, T, device=device) if args.records else None
    gathered = [0]

    def launch(counter, ep):
        if traj is not None:
            traj.reset()
        rp.play(T, counter, auto_reset=True, episodes=ep, record=traj)
        if traj is not None:            # actor -> learner rank: pack the launch's rows, gather them to rank 0
            packed = traj.pack()
            if dist is not None:
                from exploring_muzero_on_dog_amd import transfer as TR
                got = TR.gather_packed(packed, dst=0, spec=TR.dog_fields())
                if got is not None and ep is not None:
                    gathered[0] += sum(int(g["act"].shape[0]) for g in got)
            elif ep is not None:
                gathered[0] += int(packed["act"].shape[0])

    def step(k):
        ev[k][0].record()
        for _ in range(L):
            launch(env_steps, episodes)
        ev[k][1].record()

    for _ in range(args.warmup):        # the same calls as a timed step (record, pack and gather included)
        launch(warm, None)

    elapsed = timed_region(dist, step, args.steps)
    kernel_ms = sum(a.elapsed_time(b) for a, b in ev)
    (steps_done, kms, games), elapsed = sum_max(dist, device, [int(env_steps.sum().item()), kernel_ms,
                                                             int(episodes.sum().item())], elapsed)
    if rank != 0:
        if dist is not None:
            dist.destroy_process_group()
        return
    avg_ms = kms / (args.steps * L * world)         # per launch
    # algorithmic bytes of one launch: the state is read and written once per launch (it stays in LDS
    # across the T turns), plus the per-game step counter
    launch_bytes = args.batch * (2 * 156 + 8)   # + env_steps / episodes counters (read + write)
    achieved = launch_bytes / (avg_ms * 1e-3) / 1e9
    out = {
        "metric": "self-play env steps/sec, DOG 2v2 random legal policy (config d)",
        "value": round(steps_done / elapsed, 2), "unit": "env_steps/s", "n_gpus": world, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": round(1000 * elapsed / args.steps, 4), "higher_is_better": True,
        "scaling": "strong" if args.split else "weak", "vs_baseline": None, "dtype": "int8",
        "data": "synthetic (seeded deals, counter-RNG random legal actions)", "games_finished": int(games),
        "config": {"workload": f"DOG 4p teams, {args.batch} games/GPU, uniform random legal action per turn, "
                               f"{L} launches of {T} turns per step (state resident in LDS within a launch), finished "
                               f"games restart in place" + (", every turn recorded, packed and gathered to rank 0"
                                                            if args.records else ""), "games_per_gpu": args.batch,
                   "records": bool(args.records),
                   "turns_per_launch": T, "launches_per_step": L,
                   "parallelism": parallelism(args, world)},
        "roofline": dog_latency_model(avg_ms, args.batch, T, launch_bytes),
    }
    if args.records:
        out["records_gathered"] = int(gathered[0])
    if world == 1 and not args.no_cpu_baseline:
        out["cpu_baseline"] = dog_cpu_baseline(min(args.cpu_seconds, 15.0))
    print(json.dumps(out), flush=True)
    if dist is not None:
        dist.destroy_process_group()


def classic_cpu_baseline(seconds, sims, depth, max_steps, lanes=16):
    """SURVEY §8(d)'s CPU timing for config (c): the C++ restatement of classic Stochastic MuZero self-play
    (oracle/cpu_classic.cpp: classic-MADN env with the die thrown per turn, Repr2 / StochasticDynamicsNetwork4 /
    Pred4 fp32, mctx stochastic_muzero_policy with Dirichlet root noise, OpenMP over game lanes; checked against
    the NumPy oracle by tests/test_cpu_baseline_classic.py) on the host for `seconds`, at 1 thread and at all
    cores (game_agent_stochastic.py:52-218, muzero_classic_madn.py:464-517)."""
    from oracle import classic_madn as cm
    from oracle import classic_nets as CN
    from oracle import cpu_selfplay as CS
    C = cm.num_channels(CLASSIC_PLAYERS)
    net = CS.CpuClassicNet(CN.init_params(C, seed=0), C)
    cores, aff = cpu_cores()
    half = seconds / 2
    one = net.bench(CLASSIC_PLAYERS, cm.SELFPLAY_RULES, lanes, sims, depth, max_steps, TEMP, 0, 1, half)
    allc = net.bench(CLASSIC_PLAYERS, cm.SELFPLAY_RULES, lanes, sims, depth, max_steps, TEMP, 0, cores, half)
    v1 = one["env_steps"] / one["elapsed"]
    vn = allc["env_steps"] / allc["elapsed"]
    return {"value": round(vn, 2), "unit": "env_steps/s", "cores": cores, "kind": "port",
            "value_1core": round(v1, 2), "value_allcores": round(vn, 2), "cores_affinity": aff,
            "sims_per_s_allcores": round(allc["searches"] * sims / allc["elapsed"], 1),
            "sample": f"C++ restatement of the reference algorithm (oracle/cpu_classic.cpp, fp32 AVX2/FMA, OpenMP): "
                      f"classic-MADN {CLASSIC_PLAYERS}p teams streamed Stochastic MuZero self-play (Dirichlet 0.25 / "
                      f"0.3 root noise), {lanes} game lanes per thread, S={sims} D={depth}, {half:.0f} s at 1 thread "
                      f"({one['env_steps']} env-steps) and {half:.0f} s at {cores} threads ({allc['env_steps']} "
                      f"env-steps); affinity shows {aff} CPUs"}


def run_classic(args):
    """Config (c): classic MADN 4p teams (game_agent_stochastic.py:13-24 rules), B games per GPU played to
    the end with a 50-simulation Stochastic MuZero search per move (muz_classic_selfplay)."""
    rank, world, dist, device = setup(args)
    from exploring_muzero_on_dog_amd import game_agent_stochastic as GS
    from exploring_muzero_on_dog_amd import stochastic as ST
    from exploring_muzero_on_dog_amd import classic as CL
    C = CL.num_channels(CLASSIC_PLAYERS)
    net = ST.DeviceClassicNet(ST.init_classic_params(C, seed=0), C, device=device)
    eng = GS.StochasticSelfPlayEngine(net, args.batch, num_players=CLASSIC_PLAYERS, max_steps=args.max_steps,
                                      num_simulations=args.sims, max_depth=args.depth, device=device)
    def play(seed):
        if args.games:
            return eng.play_stream(args.games, seed=seed, temperature=TEMP)
        return eng.play(seed=seed, temperature=TEMP)

    for w in range(args.warmup):
        play(10_000 * rank + w)
        beat(f"warm-up {w + 1}/{args.warmup}")
    acc = {"steps": 0, "searches": 0, "search_ms": 0.0, "turns": 0}

    def step(k):
        buf = play(10_000 * rank + 1000 + k)
        st = eng.last_stats
        acc["steps"] += int(buf["idx"].sum().item())
        acc["searches"] += st["searches"]
        acc["search_ms"] += st["search_ms"]
        acc["turns"] += st["turns"]

    elapsed = timed_region(dist, step, args.steps)
    (steps_done, searches, search_ms, turns), elapsed = sum_max(
        dist, device, [acc["steps"], acc["searches"], acc["search_ms"], acc["turns"]], elapsed)
    if rank != 0:
        if dist is not None:
            dist.destroy_process_group()
        return
    out = {
        "metric": "self-play env steps/sec + MCTS sims/sec, classic MADN 4p teams (config c)",
        "value": round(steps_done / elapsed, 2), "unit": "env_steps/s", "n_gpus": world, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": round(1000 * elapsed / args.steps, 3), "higher_is_better": True,
        "scaling": "strong" if args.split else "weak", "vs_baseline": None, "dtype": "f32",
        "data": "synthetic (self-generated games, seeded random fp32 weights)",
        "config": {"workload": f"classic MADN {CLASSIC_PLAYERS}p teams self-play, {args.batch} games/GPU, "
                               f"Stochastic MuZero S={args.sims} D={args.depth}, max_steps={args.max_steps}"
                               + (f", {args.games} games per step streamed through the {args.batch} lanes"
                                  if args.games else ""), "games_per_step": args.games or args.batch,
                   "games_per_gpu": args.batch, "num_simulations": args.sims, "max_depth": args.depth,
                   "parallelism": parallelism(args, world)},
        "sims_per_s": round(searches * args.sims / elapsed, 1),
        "env_steps": int(steps_done), "searches": int(searches),
    }
    achieved = searches * args.sims * CLASSIC_FLOP_PER_SIM / (search_ms * 1e-3) / 1e12 if search_ms > 0 else 0.0
    out["roofline"] = {"bound": "mfma", "kernel": "k_stochastic_search", "achieved": round(achieved, 3),
                       "peak": PEAK_FP32_MFMA_TFLOPS, "unit": "TFLOP/s", "frac": round(achieved / PEAK_FP32_MFMA_TFLOPS, 4),
                       "avg_launch_ms": round(search_ms / max(1, turns), 4), "flop_per_sim": CLASSIC_FLOP_PER_SIM}
    traffic, traffic_src = measured_traffic("classic_traffic", "k_stochastic_search")
    avg_s = search_ms * 1e-3 / max(1, turns)
    out["roofline"].update({"traffic": None if traffic is None else round(traffic),
                            "traffic_achieved_tbs": None if traffic is None or avg_s <= 0 else
                            round(traffic / avg_s / 1e12, 3), "traffic_source": traffic_src})
    if world == 1 and not args.no_cpu_baseline:
        out["cpu_baseline"] = classic_cpu_baseline(min(args.cpu_seconds, 20.0), args.sims, args.depth, args.max_steps)
    print(json.dumps(out), flush=True)
    if dist is not None:
        dist.destroy_process_group()


def _train_overlapped(args, rank, world, dist, device, eng, ring, learner, net, games, stats, C, is_actor, is_learner,
                      learner_rank, A=24):
    """--workload train --overlap: pipeline.OverlappedIterations with this process's roles.  1 GPU: self-play in
    a worker thread on its own stream while the learner's graph replays on another; N ranks: actors play while
    the learner trains, then gather_packed + an async weight broadcast.  Returns the timed region's seconds."""
    import torch
    from exploring_muzero_on_dog_amd import pipeline as PL
    from exploring_muzero_on_dog_amd import transfer as TR
    s_play = torch.cuda.Stream(device=device) if is_actor else None
    # MUZ_LEARNER_PRIORITY=1: the learner's stream at the highest priority (its kernels dispatched ahead of the
    # self-play stream's when both wait for CUs; round-6 A/B, profiles/r6j_*)
    prio = -1 if os.environ.get("MUZ_LEARNER_PRIORITY") == "1" else 0
    s_learn = torch.cuda.Stream(device=device, priority=prio) if is_learner else None
    steps = {"n": 2}

    def play(g):
        with torch.cuda.stream(s_play):
            buf = eng.play_stream(games, seed=5000 + g + 7919 * rank, temperature=1.0, stream=s_play)
            stats["env_steps"] += int(buf["idx"].sum().item())
            if world > 1:
                buf = TR.pack(buf)
                s_play.synchronize()
            return buf

    def train(i):
        with torch.cuda.stream(s_learn):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(steps["n"]):
                learner.train_step_from(ring, losses=False)
            e1.record()
            e1.synchronize()
            stats["learner_ms"] += e0.elapsed_time(e1)
            stats["train_steps"] += steps["n"]

    def deliver(g, got):
        if world == 1:
            with torch.cuda.stream(s_learn):
                ring.save_games_from_buffers(got)
            return
        with torch.cuda.stream(s_learn if is_learner else torch.cuda.current_stream(device)):
            TR.deliver_to_learner(got if is_actor else None, ring, C, A, learner_rank, device=device)
        if is_learner:
            s_learn.synchronize()

    def publish(i):
        if world == 1:
            with torch.cuda.stream(s_learn):
                learner.push_to(net)
            s_learn.synchronize()
            return PL._Done()
        with torch.cuda.stream(s_learn if is_learner else torch.cuda.current_stream(device)):
            handle = TR.publish_weights(net, learner, learner_rank, async_op=True)
        if is_learner:
            s_learn.synchronize()
        return handle

    loop = PL.OverlappedIterations(is_actor=is_actor, is_learner=is_learner, play=play, train=train, deliver=deliver,
                                   publish=publish, concurrent=(world == 1))
    loop.prologue()                               # generation 0; then warm-up iterations at 2 learner steps
    if is_learner:
        # capture the learner's HIP graph before any iteration runs self-play in another thread (a capture
        # must not see the other thread's synchronising HIP calls)
        with torch.cuda.stream(s_learn):
            learner.train_step_from(ring, losses=False)
        s_learn.synchronize()
    for w in range(max(args.warmup, 1)):
        loop.step()
        beat(f"overlap warm-up {w + 1}")
    stats.update(env_steps=0, train_steps=0, learner_ms=0.0)
    steps["n"] = args.train_steps

    def timed(k):
        loop.step()
        if k == args.steps - 1:
            loop.finish()
    return timed_region(dist, timed, args.steps)


class _DogActor:
    """The DOG actor of the train workload: game_agent_dog.DogSelfPlay's recorded stream with SelfPlayEngine's
    play_stream signature (the stream argument: the records are written on the current torch stream)."""

    def __init__(self, net, games, T, S, D, device):
        from exploring_muzero_on_dog_amd import game_agent_dog as GAD
        self.sp = GAD.DogSelfPlay(net, games, S, D, 1.0, seed=0, device=device)
        self.games, self.T = games, T

    def play_stream(self, num_games, seed, temperature=1.0, stream=None):
        return self.sp.play_stream(num_games, self.T, temperature=temperature, seed=seed)


def run_train(args):
    """Config (e): the training loop at its reference hyper-parameters -- --game det: train_with_reward.py:167-311
    (det-MADN 4 players); --game dog: MuZero_DOG/train.py:168-300 with its config 311-352 (4p DOG teams, the DOG slice's
    nets at A = 806, its loss = train_with_reward.py's) -- 1500 games per iteration (S=100, D=50, max_len 550), replay
    ring 20000 x 550, batch 128, unroll 10, td 50, 2500 learner steps per iteration.  One bench step = one iteration.
    1 GPU: actor and learner share it.  N GPUs: ranks 0..N-2 are actors (the games split between them,
    packed and gathered to the learner over RCCL point-to-point), rank N-1 is the learner, which
    broadcasts the new weights back (one collective) -- SURVEY §8(e)."""
    import numpy as np
    import torch
    rank, world, dist, device = setup(args)
    from exploring_muzero_on_dog_amd import detmadn as E
    from exploring_muzero_on_dog_amd import game_agent as GA
    from exploring_muzero_on_dog_amd import learner as LR
    from exploring_muzero_on_dog_amd import nets as N
    from exploring_muzero_on_dog_amd import replay as R
    from exploring_muzero_on_dog_amd import transfer as TR
    dog = args.game == "dog"
    P, GAMES, T, S, D = 4, 1500, 550, 100, 50
    learner_rank = world - 1
    actors = max(world - 1, 1)
    is_actor = world == 1 or rank != learner_rank
    is_learner = world == 1 or rank == learner_rank
    games = (GAMES + actors - 1) // actors
    if dog:
        from exploring_muzero_on_dog_amd import muzero_dog as MD
        C, A = MD.NUM_CHANNELS, MD.NUM_ACTIONS
        params = MD.init_muzero_params(0)                       # MuZero_DOG/train.py:326 seed 0
        net = MD.DeviceDogNet(params, device=device)
        eng = _DogActor(net, games, T, S, D, device) if is_actor else None
        learner = LR.DogLearner(params, unroll_steps=10, device=device, graph=True) if is_learner else None
    else:
        C, A = E.num_channels(P), 24
        params = N.init_muzero_params(42, C)
        net = N.DeviceNet(params, C, device=device)
        eng = GA.SelfPlayEngine(net, games, num_players=P, max_steps=T, num_simulations=S, max_depth=D,
                                device=device) if is_actor else None
        learner = LR.Learner(params, C, unroll_steps=10, device=device, graph=True) if is_learner else None
    ring = R.VectorizedReplayBuffer(20000, 128, 10, 50, obs_shape=(C, 56), action_dim=A, max_episode_length=T,
                                    device=device, rng=np.random.RandomState(rank)) if is_learner else None
    stats = {"env_steps": 0, "train_steps": 0, "learner_ms": 0.0}

    def iteration(seed, train_steps):
        buf = eng.play_stream(games, seed=seed + 7919 * rank, temperature=1.0) if is_actor else None
        if is_actor:
            stats["env_steps"] += int(buf["idx"].sum().item())
        if world == 1:
            ring.save_games_from_buffers(buf)
        else:
            TR.deliver_to_learner(TR.pack(buf) if is_actor else None, ring, C, A, learner_rank, device=device)
        if is_learner:
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(train_steps):
                learner.train_step_from(ring, losses=False)
            e1.record()
            e1.synchronize()
            stats["learner_ms"] += e0.elapsed_time(e1)
            stats["train_steps"] += train_steps
            if world == 1:
                learner.push_to(net)
        if world > 1:
            TR.publish_weights(net, learner, learner_rank)

    if args.overlap:
        elapsed = _train_overlapped(args, rank, world, dist, device, eng, ring, learner, net, games, stats, C,
                                    is_actor, is_learner, learner_rank, A)
    else:
        for w in range(max(args.warmup, 1)):       # fills the ring and captures the learner's HIP graph
            iteration(100 * w, 2)
            beat(f"warm-up {w + 1}")
        stats.update(env_steps=0, train_steps=0, learner_ms=0.0)
        elapsed = timed_region(dist, lambda k: iteration(1000 + k, args.train_steps), args.steps)
    (env_steps, train_steps, learner_ms), elapsed = sum_max(
        dist, device, [stats["env_steps"], stats["train_steps"], stats["learner_ms"]], elapsed)
    if rank != 0:
        if dist is not None:
            dist.destroy_process_group()
        return
    flop_step = DOG_LEARNER_FLOP_PER_STEP if dog else LEARNER_FLOP_PER_STEP
    out = {
        "metric": ("MuZero training iterations/sec, DOG 2v2 (config e as BASELINE names it: the MuZero_DOG train loop, "
                   "self-play + replay + learner)" if dog else
                   "MuZero training iterations/sec, det-MADN 4p (config e: self-play + replay + learner)"),
        "value": round(args.steps / elapsed, 5), "unit": "iterations/s", "n_gpus": world, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": round(1000 * elapsed / args.steps, 1), "higher_is_better": True,
        "scaling": "strong", "vs_baseline": None, "dtype": "f32",
        "data": "synthetic (self-generated games, seeded random fp32 weights)",
        "config": {"workload": (f"MuZero_DOG/train.py config: 4p DOG teams, the DOG slice's nets (A = 806), "
                                if dog else "train_with_reward.py config: ") +
                               f"{GAMES} games/iter (S={S}, D={D}, max_len {T}), "
                               f"ring 20000, batch 128, unroll 10, td 50, {args.train_steps} learner steps/iter",
                   "game": args.game,
                   "parallelism": ("1 GPU (actor + learner)" if world == 1 else
                                   f"{world - 1} actor ranks + 1 learner rank (packed-trajectory gather, weight "
                                   f"broadcast)"),
                   "schedule": ("overlapped: iteration i+1's self-play runs while iteration i trains; games played "
                                "with weights one iteration staler than the reference's sequential loop"
                                if args.overlap else "sequential, as " +
                                ("MuZero_DOG/train.py:243-276" if dog else "train_with_reward.py:244-292"))},
        "env_steps_per_s": round(env_steps / elapsed, 1), "train_steps_per_s": round(train_steps / elapsed, 2),
    }
    if train_steps:
        step_ms = learner_ms / train_steps
        achieved = flop_step / (step_ms * 1e-3) / 1e12
        out["roofline"] = {"bound": "mfma", "kernel": "learner train_step (forward + backward + AdamW, one HIP graph)",
                           "achieved": round(achieved, 3), "peak": PEAK_FP32_MFMA_TFLOPS, "unit": "TFLOP/s",
                           "frac": round(achieved / PEAK_FP32_MFMA_TFLOPS, 5), "avg_step_ms": round(step_ms, 3),
                           "flop_per_step": flop_step,
                           "note": "batch 128 x unroll 10 of 256-wide fp32 layers: hundreds of small GEMMs and "
                                   "LayerNorms per step, latency-bound, not MFMA-bound", "traffic": None}
    print(json.dumps(out), flush=True)
    if dist is not None:
        dist.destroy_process_group()


ENV_ROUNDS_PER_STEP = 100      # --workload env: one bench step = 100 random-play env rounds (one launch each)
# csrc/env_detmadn.hip launch_det_round: the kernel variant 0 picks by batch size (one game per 32 lanes up to
# 2^13 games, per 4 lanes up to 2^16, per lane above)
def env_auto_variant(B):
    return 2 if B <= (1 << 13) else 4 if B <= (1 << 16) else 1
ENV_PREROLL = 300              # rounds played before warm-up: games spread over 0..300 plies (SURVEY §8(d)(b'))


def env_bytes_per_step(P):
    """Algorithmic HBM bytes of one env-step of muz_detmadn_random_round: the SoA state read and
    written (board 56 + pins 4P + current player, reward, done + action set 6P), the legal mask read and
    written, reward and done written, and the int8 observation (8P+2) x 56 written.  2p: 1176 B."""
    state = 56 + 4 * P + 3 + 6 * P
    return 2 * state + 2 * 4 + 2 + (8 * P + 2) * 56


def measured_env_traffic(B, kernel):
    """HBM bytes per env-round launch from the newest committed PMC summary of this batch
    (profiles/r*_env_pmc_<B>.json, profiles/summarize_env_pmc.py: FETCH_SIZE doubled per the gfx950 note + WRITE_SIZE).
    Returns (bytes, source) or (None, None)."""
    import glob
    for f in sorted(glob.glob(os.path.join(ROOT, "profiles", f"r*_env_pmc_{B}.json")), reverse=True):
        t = json.load(open(f))
        if t.get("kernel", kernel) == kernel and "hbm_bytes_per_launch" in t:
            return t["hbm_bytes_per_launch"], os.path.relpath(f, ROOT)
    return None, None


def run_env(args):
    """SURVEY §8(d)(b'): the env kernels alone -- step + legal + encode of det-MADN 2p over the batch -- as the
    fused random-play round (muz_detmadn_random_round), on a mid-game state distribution (ENV_PREROLL rounds
    of seeded random legal play first; finished games restart in place).  One bench step = 100 rounds."""
    import torch
    rank, world, dist, device = setup(args)
    from exploring_muzero_on_dog_amd import detmadn as E
    B, R = args.batch, ENV_ROUNDS_PER_STEP
    env = E.env_reset(B, num_players=PLAYERS, device=device, **E.SELFPLAY_RULES)
    legal = E.legal_bits(env)
    C = E.num_channels(PLAYERS)
    obs = torch.empty((B, C, E.CELLS), dtype=torch.int8, device=device)
    reward = torch.empty(B, dtype=torch.int8, device=device)
    done = torch.empty(B, dtype=torch.uint8, device=device)
    seed = 77 + 1000 * rank
    turn = [0]

    def rounds(k, ev=None):
        for i in range(R):
            if ev is not None:
                ev[2 * (k * R + i)].record()
            E.random_round(env, legal, seed, turn[0], obs=obs, reward=reward, done=done, variant=args.env_variant)
            if ev is not None:
                ev[2 * (k * R + i) + 1].record()
            turn[0] += 1

    for _ in range(ENV_PREROLL // R):
        rounds(0)
    for _ in range(args.warmup):
        rounds(0)
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2 * R * args.steps)]
    elapsed = timed_region(dist, lambda k: rounds(k, ev), args.steps)
    launch_ms = sum(ev[2 * i].elapsed_time(ev[2 * i + 1]) for i in range(R * args.steps))
    (steps_done, lms), elapsed = sum_max(dist, device, [B * R * args.steps, launch_ms], elapsed)
    if rank != 0:
        if dist is not None:
            dist.destroy_process_group()
        return
    avg_ms = lms / (R * args.steps * world)
    per = env_bytes_per_step(PLAYERS)
    variant = args.env_variant or env_auto_variant(B)
    kernel = {1: "k_det_round", 2: "k_det_round_g<32>", 3: "k_det_round_g<8>", 4: "k_det_round_g<4>",
              5: "k_det_round_g<16>"}[variant]
    achieved = B * per / (avg_ms * 1e-3) / 1e9
    out = {
        "metric": "env-only steps/sec (step + legal + encode), det-MADN 2p random legal play (SURVEY 8(d)(b'))",
        "value": round(steps_done / elapsed, 1), "unit": "env_steps/s", "n_gpus": world, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": round(1000 * elapsed / args.steps, 3), "higher_is_better": True,
        "scaling": "strong" if args.split else "weak", "vs_baseline": None, "dtype": "int8",
        "data": "synthetic (seeded random legal play, counter RNG)",
        "config": {"workload": f"det-MADN {PLAYERS}p env rounds: {B} games/GPU, {R} rounds per step, each one "
                               f"muz_detmadn_random_round launch (legal -> random legal action -> env_step / no_step "
                               f"-> reset finished -> next legal + int8 obs), after {ENV_PREROLL} pre-roll rounds",
                   "games_per_gpu": B, "rounds_per_step": R, "kernel": kernel, "parallelism": parallelism(args, world)},
        "roofline": {"bound": "hbm", "kernel": kernel, "achieved": round(achieved, 1), "peak": PEAK_HBM_GBS,
                     "unit": "GB/s", "frac": round(achieved / PEAK_HBM_GBS, 4), "avg_launch_ms": round(avg_ms, 5),
                     "bytes_per_env_step": per, "bytes_per_launch": B * per, "traffic": None},
    }
    traffic, src = measured_env_traffic(B, kernel)
    if traffic:
        out["roofline"].update(traffic=round(traffic), traffic_unit="bytes/launch (HBM, PMC)", traffic_source=src,
                               traffic_over_algorithmic=round(traffic / (B * per), 3))
    if world == 1 and not args.no_cpu_baseline:
        from oracle import cpu_selfplay as CS
        cores, aff = cpu_cores()
        half = min(args.cpu_seconds, 20.0) / 2
        s1, t1 = CS.env_bench(PLAYERS, E.SELFPLAY_RULES, 1024, 1, 1, half)
        sn, tn = CS.env_bench(PLAYERS, E.SELFPLAY_RULES, 1024, 1, cores, half)
        out["cpu_baseline"] = {"value": round(sn / tn, 1), "unit": "env_steps/s", "cores": cores, "kind": "port",
                               "value_1core": round(s1 / t1, 1), "value_allcores": round(sn / tn, 1),
                               "cores_affinity": aff,
                               "sample": f"C++ restatement (oracle/cpu_selfplay.cpp muzcpu_env_bench): 1024 games per "
                                         f"thread of random-play rounds incl. fp32 encode, {half:.0f} s at 1 thread "
                                         f"and {half:.0f} s at {cores} threads"}
    print(json.dumps(out), flush=True)
    if dist is not None:
        dist.destroy_process_group()


def run_selftest(args):
    """CPU rehearsal of the multi-rank plumbing (launcher, barrier + timed region, sum / max reduction,
    rank-0 JSON) without a GPU: each rank 'processes' (rank + 1) x batch units per step.  Only for
    tests/test_bench_launcher.py (MUZ_BENCH_BACKEND=gloo)."""
    rank, world, dist, device = setup(args)
    done = {"units": 0}

    def step(k):
        time.sleep(0.01 * (rank + 1))
        done["units"] += (rank + 1) * args.batch

    elapsed = timed_region(dist, step, args.steps)
    (units,), elapsed = sum_max(dist, device, [done["units"]], elapsed)
    if rank == 0:
        print(json.dumps({"metric": "launcher selftest", "value": units / elapsed, "unit": "units/s",
                          "n_gpus": world, "steps": args.steps, "warmup": args.warmup, "units": int(units),
                          "elapsed": elapsed, "scaling": "strong" if args.split else "weak",
                          "config": {"games_per_gpu": args.batch, "parallelism": parallelism(args, world)}}),
              flush=True)
    if dist is not None:
        dist.destroy_process_group()


def run_det(args):
    """Config (b), the BASELINE.json headline: det-MADN 2p self-play, 4096 concurrent games per GPU (or the
    job's 4096 split over the ranks with --split), Gumbel MuZero S=50 D=25."""
    import torch
    rank, world, dist, device = setup(args)
    from exploring_muzero_on_dog_amd import game_agent as GA
    from exploring_muzero_on_dog_amd import nets as N
    from exploring_muzero_on_dog_amd import detmadn as E

    C = E.num_channels(PLAYERS)
    net = N.DeviceNet(N.init_muzero_params(0, C), C, device=device)
    eng = GA.SelfPlayEngine(net, args.batch, num_players=PLAYERS, max_steps=args.max_steps,
                            num_simulations=args.sims, max_depth=args.depth, device=device)

    def play(seed):
        if args.games:
            return eng.play_stream(args.games, seed=seed, temperature=TEMP)
        return eng.play(seed=seed, temperature=TEMP)

    for w in range(args.warmup):
        play(10_000 * rank + w)
        beat(f"warm-up {w + 1}/{args.warmup}")
    torch.cuda.synchronize()
    acc = {"steps": 0, "searches": 0, "search_ms": 0.0, "launches": 0}

    def step(k):
        buf = play(10_000 * rank + 1000 + k)
        st = eng.last_stats
        acc["steps"] += int(buf["idx"].sum().item())
        acc["searches"] += st["searches"]
        acc["search_ms"] += st["search_ms"]
        acc["launches"] += st["turns"]

    elapsed = timed_region(dist, step, args.steps)
    (steps_done, searches, search_ms, launches), elapsed = sum_max(
        dist, device, [acc["steps"], acc["searches"], acc["search_ms"], acc["launches"]], elapsed)
    # Secondary figure in the reference's own loop shape (game_agent.py:185-192): ONE play_n_games_v3 batch of
    # --batch games per rank played to completion (the batch shrinks as games finish), timed on its own after
    # the K streamed steps; `value` stays the streamed rate.
    single = {"steps": 0}

    def single_batch(_):
        single["steps"] += int(eng.play(seed=10_000 * rank + 999, temperature=TEMP)["idx"].sum().item())

    single_elapsed = timed_region(dist, single_batch, 1) if args.games else None
    if single_elapsed is not None:
        (single_steps,), single_elapsed = sum_max(dist, device, [single["steps"]], single_elapsed)
    if rank != 0:
        if dist is not None:
            dist.destroy_process_group()
        return
    value = steps_done / elapsed
    # roofline of the dominant kernel (k_gumbel_search): algorithmic FLOP / HIP-event time of its launches
    traffic, traffic_src = measured_traffic()
    flop = searches * args.sims * FLOP_PER_SIM
    achieved = flop / (search_ms * 1e-3) / 1e12 if search_ms > 0 else 0.0
    out = {
        "metric": "self-play env steps/sec + MCTS sims/sec, det-MADN batch=4096, 1/2/4/8 GPU",
        "value": round(value, 2),
        "unit": "env_steps/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(1000 * elapsed / args.steps, 3),
        "higher_is_better": True,
        "scaling": "strong" if args.split else "weak",
        "vs_baseline": None,
        "dtype": "f32",
        "data": "synthetic (self-generated games, seeded random fp32 weights)",
        "config": {"workload": f"det-MADN {PLAYERS}p self-play, {args.batch} games/GPU, Gumbel MuZero "
                               f"S={args.sims} D={args.depth}, max_steps={args.max_steps}, temp={TEMP}"
                               + (f", {args.games} games per step per GPU streamed through the {args.batch} lanes"
                                  if args.games else ""),
                   "games_per_gpu": args.batch, "job_batch": args.job_batch if args.split else args.batch * world,
                   "games_per_step": (args.games or args.batch) * world,
                   "num_simulations": args.sims, "max_depth": args.depth,
                   "parallelism": parallelism(args, world)},
        "sims_per_s": round(searches * args.sims / elapsed, 1),
        "value_single_batch": (round(single_steps / single_elapsed, 2) if single_elapsed else round(value, 2)),
        "single_batch": ({"games_per_gpu": args.batch, "env_steps": int(single_steps),
                          "seconds": round(single_elapsed, 4), "unit": "env_steps/s",
                          "what": "one play_n_games_v3 batch per rank to completion (game_agent.py:185-192), "
                                  "timed after the streamed steps"} if single_elapsed else
                         {"what": "--games 0: value itself is the single-batch rate"}),
        "env_steps": int(steps_done),
        "searches": int(searches),
        "roofline": {"bound": "mfma", "kernel": "k_gumbel_search", "achieved": round(achieved, 3),
                     "peak": PEAK_FP32_MFMA_TFLOPS, "unit": "TFLOP/s",
                     "frac": round(achieved / PEAK_FP32_MFMA_TFLOPS, 4),
                     # the same algorithmic FLOP over the whole wall clock (root inference, env kernels, host gaps)
                     "end_to_end_frac": round(searches * args.sims * FLOP_PER_SIM / elapsed / 1e12
                                              / PEAK_FP32_MFMA_TFLOPS / world, 4),
                     "avg_launch_ms": round(search_ms / max(1, launches), 4),
                     "flop_per_sim": FLOP_PER_SIM, "executed_flop_per_sim": EXEC_FLOP_PER_SIM,
                     "executed_frac": round(achieved * EXEC_FLOP_PER_SIM / FLOP_PER_SIM / PEAK_FP32_MFMA_TFLOPS, 4),
                     "traffic": traffic, "traffic_unit": "bytes/launch (HBM, PMC)", "traffic_source": traffic_src},
    }
    l2, mfma_busy, l2_src = measured_l2_reads()
    if l2 and launches:
        avg_s = search_ms / launches * 1e-3
        # second ceiling: the weights stream from L2 every simulation (a 16-row tile reuses each weight byte
        # for 8 FLOP); at the L2-served rate the launch could not be shorter than l2 / 18.8 TB/s
        out["roofline"]["l2_stream"] = {"bytes_per_launch": round(l2), "achieved_TBs": round(l2 / avg_s / 1e12, 2),
                                        "ceiling_TBs": L2_SERVED_TBS, "frac": round(l2 / avg_s / 1e12 / L2_SERVED_TBS, 4),
                                        "mfma_frac_at_l2_ceiling": round(achieved / PEAK_FP32_MFMA_TFLOPS * avg_s /
                                                                         (l2 / (L2_SERVED_TBS * 1e12)), 4),
                                        "source": l2_src}
    if mfma_busy is not None:
        out["roofline"]["mfma_busy_frac"] = {"value": round(mfma_busy, 4), "counter": "SQ_VALU_MFMA_BUSY_CYCLES / "
                                             "(GRBM_GUI_ACTIVE / 8 x 256 CUs x 4 SIMDs)", "source": l2_src}
    loop = measured_loop_ceiling()
    if loop:
        out["roofline"]["loop_ceiling"] = dict(loop, frac_of_ceiling=round(achieved / PEAK_FP32_MFMA_TFLOPS / loop["frac"], 4))
    if world == 1 and not args.no_cpu_baseline:
        out["cpu_baseline"] = cpu_baseline(args.cpu_seconds, args.sims, args.depth, args.max_steps)
    print(json.dumps(out), flush=True)
    if dist is not None:
        dist.destroy_process_group()


def main():
    args = parse()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(launch_ranks(args.gpus))
    if args.workload == "dog" and args.policy == "muzero":
        return run_dog_muzero(args)
    return {"train": run_train, "dog": run_dog, "classic": run_classic, "det": run_det, "env": run_env,
            "selftest": run_selftest}[args.workload](args)


if __name__ == "__main__":
    main()
