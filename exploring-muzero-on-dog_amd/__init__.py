"""MI355X-native MuZero self-play engine for the MADN / DOG games.

Host side of libmuz.so (include/muz.h).  Mirrors the reference's entry points:
  * ``detmadn``   -- MADN/deterministic_madn.py env API (batched, device-resident SoA)
  * ``nets``      -- MuZero_det_MADN/muzero_deterministic_madn.py networks
  * ``mcts``      -- run_muzero_mcts (Gumbel MuZero search, mctx 0.0.6 semantics)
  * ``game_agent``-- MuZero_det_MADN/game_agent.py self-play driver
Everything on the compute path runs in hand-written HIP kernels; importing a module
whose kernels are missing raises instead of falling back to CPU code.
"""
__all__ = ["detmadn", "nets", "mcts", "game_agent", "lib"]
