"""ctypes binding of libmuz.so (C ABI declared in include/muz.h).

No torch types cross the boundary: callers pass raw device pointers
(``tensor.data_ptr()``) and a ``hipStream_t`` (``torch.cuda.current_stream().cuda_stream``).
There is deliberately no CPU fallback: if the library is missing this module raises.
"""
import ctypes
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
# MUZ_LIB selects an alternative build (e.g. the stamp-instrumented libmuz_diag.so); default in-tree.
LIB_PATH = os.environ.get("MUZ_LIB") or os.path.join(_HERE, "libmuz.so")

c_i8p = ctypes.POINTER(ctypes.c_int8)
c_u8p = ctypes.POINTER(ctypes.c_uint8)
vp = ctypes.c_void_p

MUZ_OK = 0
MUZ_E_BASE = 10000
MUZ_E_INVALID = MUZ_E_BASE + 1
MUZ_E_UNSUPPORTED = MUZ_E_BASE + 2


class MuzRuleAgent(ctypes.Structure):
    _fields_ = [("temperature", ctypes.c_float), ("goal_bonus", ctypes.c_float), ("out_many", ctypes.c_float),
                ("out_few", ctypes.c_float), ("hit_bonus", ctypes.c_float)]


class MuzDogTraj(ctypes.Structure):
    _fields_ = [("act", ctypes.c_void_p), ("player", ctypes.c_void_p), ("reward", ctypes.c_void_p),
                ("legal", ctypes.c_void_p), ("done", ctypes.c_void_p), ("idx", ctypes.c_void_p),
                ("max_steps", ctypes.c_int32)]


class MuzWgradProblem(ctypes.Structure):
    _fields_ = [("x", vp), ("dz", vp), ("out", vp)] + [(k, ctypes.c_int32) for k in ("M", "K", "N", "ldx", "lddz")]


class MuzColsumProblem(ctypes.Structure):
    _fields_ = [("src", vp), ("out0", vp), ("out1", vp), ("out2", vp)] + \
        [(k, ctypes.c_int32) for k in ("kind", "rows", "N", "ld")]


class MuzTransposeProblem(ctypes.Structure):
    _fields_ = [("src", vp), ("dst", vp), ("K", ctypes.c_int32), ("N", ctypes.c_int32), ("ldt", ctypes.c_int32)]


MUZ_CHAIN_MAX_T = 32


class MuzChainGroup(ctypes.Structure):
    """muz_chain_group (include/muz.h): one trunk's parameters and stacked buffers for muz_trunk_chain_*."""
    _fields_ = [("ln0_gamma", vp), ("ln0_beta", vp), ("wf", vp * 7), ("wb", vp * 7), ("bias", vp * 7), ("gamma", vp * 6),
                ("beta", vp * 6), ("X", vp * 7), ("DZ", vp * 7), ("part", vp * 7)]


class MuzChainArgs(ctypes.Structure):
    _fields_ = [("T", ctypes.c_int32), ("M", ctypes.c_int32), ("ngroups", ctypes.c_int32),
                ("app", ctypes.c_int32 * MUZ_CHAIN_MAX_T), ("slot", ctypes.c_int32 * MUZ_CHAIN_MAX_T),
                ("scaled", ctypes.c_int32 * MUZ_CHAIN_MAX_T), ("group", MuzChainGroup * 2), ("latent0", vp),
                ("scale1", vp), ("shift", vp), ("out", vp), ("q", vp), ("lohi", vp), ("idx", vp), ("ln0_out", vp),
                ("z", vp), ("stats", vp), ("g", vp), ("h", vp), ("grad_scale", ctypes.c_float), ("dscale", vp),
                ("dshift", vp), ("dlatent0", vp), ("out_twin", vp), ("stack0", vp), ("g0", vp)]


MUZ_RBSTACK_MAX = 6


class MuzRbstackArgs(ctypes.Structure):
    """muz_rbstack_args (include/muz.h): a stack of ResBlocks for muz_rbstack_fwd / _bwd."""
    _L = 2 * MUZ_RBSTACK_MAX
    _fields_ = [("nb", ctypes.c_int32), ("M", ctypes.c_int32), ("wf", vp * _L), ("wb", vp * _L), ("bias", vp * _L),
                ("gamma", vp * _L), ("beta", vp * _L), ("x", vp), ("X", vp), ("out", vp), ("z", vp), ("stats", vp),
                ("g", vp), ("DZ", vp), ("part", vp), ("dx", vp)]


class MuzLossTerm(ctypes.Structure):
    _fields_ = [("logits", vp), ("dlogits", vp), ("labels", vp), ("probs", vp), ("ncls", ctypes.c_int32),
                ("ld", ctypes.c_int32), ("rare_not_one", ctypes.c_int32), ("w_rare", ctypes.c_float),
                ("w_common", ctypes.c_float), ("scale", ctypes.c_float)]


class MuzHeadsArgs(ctypes.Structure):
    _fields_ = [(k, ctypes.c_int32) for k in ("R", "Rk", "A")] + [(k, vp) for k in (
        "pol_h", "v_h", "head_in", "onehot", "W2", "b2", "W4", "b4", "W5", "b5", "W6", "b6", "Wr", "br", "W7", "b7",
        "Wd", "bd", "logits", "value", "h4", "rl", "dl", "h6", "h7", "ri", "g_logits", "g_value", "g_rl", "g_dl",
        "d_pol_h", "d_v_h", "d_head_in", "dz4", "dv5", "dz6", "dz7")]


class MuzLossArgs(ctypes.Structure):
    _fields_ = [(k, ctypes.c_int32) for k in ("K", "B", "A", "T", "nterms", "norm")] + \
        [(k, vp) for k in ("masks", "target_values", "policies", "value", "logits", "dvalue", "dlogits")] + \
        [("scale_value", ctypes.c_float), ("scale_policy", ctypes.c_float), ("term", MuzLossTerm * 3),
         ("parts", vp), ("total", vp), ("partials", vp), ("ticket", vp)]


class MuzRules(ctypes.Structure):
    _fields_ = [
        ("num_players", ctypes.c_int32),
        ("distance", ctypes.c_int32),
        ("layout", ctypes.c_int32 * 4),
        ("starting_player", ctypes.c_int32),
        ("enable_teams", ctypes.c_int32),
        ("enable_initial_free_pin", ctypes.c_int32),
        ("enable_circular_board", ctypes.c_int32),
        ("enable_start_blocking", ctypes.c_int32),
        ("enable_jump_in_goal_area", ctypes.c_int32),
        ("enable_friendly_fire", ctypes.c_int32),
        ("enable_start_on_1", ctypes.c_int32),
        ("enable_bonus_turn_on_6", ctypes.c_int32),
        ("must_traverse_start", ctypes.c_int32),
        ("enable_dice_rethrow", ctypes.c_int32),
        ("disable_swapping", ctypes.c_int32),
        ("disable_hot_seven", ctypes.c_int32),
        ("disable_joker", ctypes.c_int32),
    ]


class MuzDogSoA(ctypes.Structure):
    _fields_ = [(k, vp) for k in ("board", "pins", "deck", "hands", "swap_choices", "current_player",
                                  "round_starter", "phase", "hand_size", "reward", "done", "deal")] + [
        ("stride", ctypes.c_int32)]


class MuzTttState(ctypes.Structure):
    _fields_ = [("board", ctypes.c_int8 * 9), ("current_player", ctypes.c_int8), ("reward", ctypes.c_int8),
                ("done", ctypes.c_uint8), ("memory", ctypes.c_int8 * 6)]


class MuzTttPolicyOut(ctypes.Structure):
    _fields_ = [("action", ctypes.c_int32), ("visits", ctypes.c_int32 * 9), ("action_weights", ctypes.c_double * 9),
                ("value", ctypes.c_double)]


class MuzDetSoA(ctypes.Structure):
    _fields_ = [
        ("board", vp),
        ("pins", vp),
        ("current_player", vp),
        ("reward", vp),
        ("done", vp),
        ("action_set", vp),
        ("stride", ctypes.c_int32),
    ]


class MuzClassicSoA(ctypes.Structure):
    _fields_ = [
        ("board", vp),
        ("pins", vp),
        ("current_player", vp),
        ("reward", vp),
        ("done", vp),
        ("die", vp),
        ("stride", ctypes.c_int32),
    ]


class MuzDense(ctypes.Structure):
    _fields_ = [("w", vp), ("b", vp)]


class MuzLn(ctypes.Structure):
    _fields_ = [("scale", vp), ("bias", vp)]


class MuzResblock(ctypes.Structure):
    _fields_ = [("d0", MuzDense), ("ln0", MuzLn), ("d1", MuzDense), ("ln1", MuzLn)]


class MuzReprW(ctypes.Structure):
    _fields_ = [("conv0", MuzDense), ("ln0", MuzLn), ("conv1", MuzDense), ("ln1", MuzLn), ("conv2", MuzDense),
                ("ln2", MuzLn), ("d0", MuzDense), ("ln3", MuzLn), ("d1", MuzDense), ("ln4", MuzLn),
                ("d2", MuzDense), ("ln5", MuzLn), ("d3", MuzDense), ("ln6", MuzLn), ("rb", MuzResblock * 6),
                ("d4", MuzDense)]


class MuzDynW(ctypes.Structure):
    _fields_ = [("d0", MuzDense), ("ln0", MuzLn), ("d12", MuzDense), ("d3", MuzDense), ("ln1", MuzLn),
                ("d4", MuzDense), ("ln2", MuzLn), ("rb", MuzResblock * 2), ("d5", MuzDense), ("d67", MuzDense),
                ("d67_onehot", vp), ("reward_head", MuzDense), ("discount_head", MuzDense),
                ("film", vp)]


class MuzPredW(ctypes.Structure):
    _fields_ = [("ln0", MuzLn), ("rb", MuzResblock * 2), ("d03", MuzDense), ("ln1", MuzLn), ("d1", MuzDense),
                ("ln2", MuzLn), ("d2", MuzDense), ("ln3", MuzLn), ("d4", MuzDense), ("d5", MuzDense)]


class MuzNetW(ctypes.Structure):
    _fields_ = [("obs_channels", ctypes.c_int32), ("num_actions", ctypes.c_int32), ("repr", MuzReprW),
                ("dyn", MuzDynW), ("pred", MuzPredW)]



class MuzDogNetW(ctypes.Structure):
    _fields_ = [("obs_channels", ctypes.c_int32), ("num_actions", ctypes.c_int32), ("repr", MuzReprW),
                ("repr_ln7", MuzLn), ("dyn", MuzDynW), ("pred", MuzPredW), ("logits", MuzDense * 4)]


class MuzSdynW(ctypes.Structure):
    _fields_ = [("act_embed", MuzDense), ("act_input_ln", MuzLn), ("act_film", MuzDense), ("act_dense1", MuzDense),
                ("act_ln1", MuzLn), ("act_dense2", MuzDense), ("act_ln2", MuzLn), ("act_rb", MuzResblock * 2),
                ("act_proj", MuzDense), ("rc", MuzDense), ("reward_onehot", vp), ("reward_head", MuzDense),
                ("discount_dense", MuzDense), ("discount_ln", MuzLn), ("discount_head", MuzDense),
                ("chance_embed", MuzDense), ("chance_input_ln", MuzLn), ("chance_film", MuzDense),
                ("chance_dense1", MuzDense), ("chance_ln1", MuzLn), ("chance_dense2", MuzDense), ("chance_ln2", MuzLn),
                ("chance_rb", MuzResblock * 2), ("chance_proj", MuzDense), ("act_film_tab", vp),
                ("chance_film_tab", vp)]


class MuzClassicNetW(ctypes.Structure):
    _fields_ = [("obs_channels", ctypes.c_int32), ("num_actions", ctypes.c_int32), ("repr", MuzReprW),
                ("sdyn", MuzSdynW), ("pred", MuzPredW)]


class MuzStochCfg(ctypes.Structure):
    _fields_ = [("num_simulations", ctypes.c_int32), ("max_depth", ctypes.c_int32),
                ("dirichlet_fraction", ctypes.c_float), ("dirichlet_alpha", ctypes.c_float),
                ("pb_c_init", ctypes.c_float), ("pb_c_base", ctypes.c_float), ("temperature", ctypes.c_float),
                ("turn", ctypes.c_int32), ("seed", ctypes.c_uint64)]


class MuzSearchCfg(ctypes.Structure):
    _fields_ = [("num_simulations", ctypes.c_int32), ("max_depth", ctypes.c_int32),
                ("max_num_considered", ctypes.c_int32), ("value_scale", ctypes.c_float),
                ("maxvisit_init", ctypes.c_float), ("gumbel_scale", ctypes.c_float), ("seed", ctypes.c_uint64),
                ("turn", ctypes.c_int32)]


class MuzTraj(ctypes.Structure):
    _fields_ = [("obs", vp), ("act", vp), ("rew", vp), ("val", vp), ("pol", vp), ("mask", vp), ("player", vp),
                ("team", vp), ("discount", vp), ("idx", vp), ("max_steps", ctypes.c_int32)]


class MuzRing(ctypes.Structure):
    _fields_ = [("obs", vp), ("act", vp), ("rew", vp), ("val", vp), ("pol", vp), ("mask", vp), ("player", vp),
                ("team", vp), ("discount", vp), ("ep_len", vp), ("capacity", ctypes.c_int32),
                ("max_steps", ctypes.c_int32), ("obs_channels", ctypes.c_int32), ("num_actions", ctypes.c_int32),
                ("won_if_positive", ctypes.c_int32), ("dice", vp), ("dice_dist", vp)]


class MuzSample(ctypes.Structure):
    _fields_ = [("observations", vp), ("actions", vp), ("rewards", vp), ("policies", vp), ("values", vp),
                ("masks", vp), ("target_values", vp), ("discount_targets", vp), ("dice_outcomes", vp),
                ("dice_probs", vp)]


class MuzTrajChance(ctypes.Structure):
    _fields_ = [("dice", vp), ("dice_dist", vp)]


class MuzSpStats(ctypes.Structure):
    _fields_ = [("turns", ctypes.c_int32), ("searches", ctypes.c_int64), ("search_ms", ctypes.c_double),
                ("total_ms", ctypes.c_double)]


# name -> (restype, argtypes).  Kept in sync with include/muz.h (tests/test_capi.py checks it).
SIGNATURES = {
    "muz_version": (ctypes.c_char_p, []),
    "muz_error_string": (ctypes.c_char_p, [ctypes.c_int]),
    "muz_detmadn_reset": (ctypes.c_int, [ctypes.POINTER(MuzRules), MuzDetSoA, ctypes.c_int32, vp]),
    "muz_detmadn_reset_seeded": (ctypes.c_int, [ctypes.POINTER(MuzRules), MuzDetSoA, vp, ctypes.c_int32, vp]),
    "muz_detmadn_legal": (ctypes.c_int, [ctypes.POINTER(MuzRules), MuzDetSoA, vp, ctypes.c_int32, vp]),
    "muz_detmadn_step": (ctypes.c_int, [ctypes.POINTER(MuzRules), MuzDetSoA, vp, vp, vp, vp, ctypes.c_int32, vp]),
    "muz_detmadn_step_pin_move": (ctypes.c_int, [ctypes.POINTER(MuzRules), MuzDetSoA, vp, vp, vp, vp,
                                                 ctypes.c_int32, vp]),
    "muz_detmadn_nostep": (ctypes.c_int, [ctypes.POINTER(MuzRules), MuzDetSoA, vp, vp, ctypes.c_int32, vp]),
    "muz_detmadn_encode_f32": (ctypes.c_int, [ctypes.POINTER(MuzRules), MuzDetSoA, vp, ctypes.c_int32, vp]),
    "muz_detmadn_encode_i8": (ctypes.c_int, [ctypes.POINTER(MuzRules), MuzDetSoA, vp, ctypes.c_int32, vp]),
    "muz_detmadn_random_round": (ctypes.c_int, [ctypes.POINTER(MuzRules), MuzDetSoA, vp, ctypes.c_uint64, ctypes.c_int32,
                                                vp, vp, vp, ctypes.c_int32, vp]),
    "muz_detmadn_random_round_variant": (ctypes.c_int, [ctypes.POINTER(MuzRules), MuzDetSoA, vp, ctypes.c_uint64,
                                                        ctypes.c_int32, vp, vp, vp, ctypes.c_int32, ctypes.c_int32, vp]),
    "muz_detmadn_policy_action": (ctypes.c_int, [ctypes.POINTER(MuzRules), MuzDetSoA, vp, ctypes.c_int32,
                                                 ctypes.POINTER(MuzRuleAgent), ctypes.c_uint64, ctypes.c_int32, vp, vp,
                                                 ctypes.c_int32, vp]),
    "muz_dog_reset": (ctypes.c_int, [ctypes.POINTER(MuzRules), MuzDogSoA, ctypes.c_uint64, ctypes.c_int32, vp]),
    "muz_dog_legal": (ctypes.c_int, [ctypes.POINTER(MuzRules), MuzDogSoA, vp, ctypes.c_int32, vp]),
    "muz_dog_step": (ctypes.c_int, [ctypes.POINTER(MuzRules), MuzDogSoA, vp, ctypes.c_uint64, vp, vp, ctypes.c_int32,
                                    vp]),
    "muz_dog_step_restart": (ctypes.c_int, [ctypes.POINTER(MuzRules), MuzDogSoA, vp, ctypes.c_uint64, vp, vp, vp,
                                            ctypes.c_int32, vp]),
    "muz_dog_sp_record_step": (ctypes.c_int, [ctypes.POINTER(MuzRules), MuzDogSoA, vp, vp, vp, vp, ctypes.c_uint64,
                                              MuzTraj, vp, vp, vp, ctypes.c_int32, vp]),
    "muz_dog_sp_assign": (ctypes.c_int, [vp, vp, vp, vp, ctypes.c_int32, vp]),
    "muz_dog_nostep": (ctypes.c_int, [ctypes.POINTER(MuzRules), MuzDogSoA, ctypes.c_uint64, vp, vp, ctypes.c_int32,
                                      vp]),
    "muz_dog_step_move": (ctypes.c_int, [ctypes.POINTER(MuzRules), MuzDogSoA, vp, vp, vp, vp, ctypes.c_int32, vp]),
    "muz_dog_random_turn": (ctypes.c_int, [ctypes.POINTER(MuzRules), MuzDogSoA, ctypes.c_uint64, ctypes.c_int32, vp,
                                           vp, vp, ctypes.c_int32, vp]),
    "muz_dog_random_play": (ctypes.c_int, [ctypes.POINTER(MuzRules), MuzDogSoA, ctypes.c_uint64, ctypes.c_int32,
                                           ctypes.c_int32, ctypes.c_int32, vp, vp, ctypes.c_int32, vp]),
    "muz_dog_random_play_record": (ctypes.c_int, [ctypes.POINTER(MuzRules), MuzDogSoA, ctypes.c_uint64,
                                                  ctypes.c_int32, ctypes.c_int32, ctypes.c_int32, vp, vp, MuzDogTraj,
                                                  ctypes.c_int32, vp]),
    "muz_dog_random_action": (ctypes.c_int, [vp, vp, ctypes.c_uint64, ctypes.c_int32, vp, ctypes.c_int32, vp]),
    "muz_classic_reset": (ctypes.c_int, [ctypes.POINTER(MuzRules), MuzClassicSoA, ctypes.c_int32, vp]),
    "muz_classic_reset_seeded": (ctypes.c_int, [ctypes.POINTER(MuzRules), MuzClassicSoA, vp, ctypes.c_int32, vp]),
    "muz_classic_set_die": (ctypes.c_int, [ctypes.POINTER(MuzRules), MuzClassicSoA, vp, ctypes.c_int32, vp]),
    "muz_classic_dice_probs": (ctypes.c_int, [ctypes.POINTER(MuzRules), MuzClassicSoA, vp, vp, ctypes.c_int32, vp]),
    "muz_classic_throw_die": (ctypes.c_int, [ctypes.POINTER(MuzRules), MuzClassicSoA, vp, vp, ctypes.c_int32, vp]),
    "muz_classic_legal": (ctypes.c_int, [ctypes.POINTER(MuzRules), MuzClassicSoA, vp, ctypes.c_int32, vp]),
    "muz_classic_step": (ctypes.c_int, [ctypes.POINTER(MuzRules), MuzClassicSoA, vp, vp, vp, ctypes.c_int32, vp]),
    "muz_classic_nostep": (ctypes.c_int, [ctypes.POINTER(MuzRules), MuzClassicSoA, vp, vp, ctypes.c_int32, vp]),
    "muz_classic_policy_action": (ctypes.c_int, [ctypes.POINTER(MuzRules), MuzClassicSoA, vp, ctypes.c_int32,
                                                 ctypes.POINTER(MuzRuleAgent), ctypes.c_uint64, ctypes.c_int32, vp, vp,
                                                 ctypes.c_int32, vp]),
    "muz_classic_encode_f32": (ctypes.c_int, [ctypes.POINTER(MuzRules), MuzClassicSoA, vp, ctypes.c_int32, vp]),
    "muz_classic_encode_i8": (ctypes.c_int, [ctypes.POINTER(MuzRules), MuzClassicSoA, vp, ctypes.c_int32, vp]),
    "muz_tile_waves": (ctypes.c_int32, []),
    "muz_ttt_reset": (ctypes.c_int, [ctypes.POINTER(MuzTttState)]),
    "muz_ttt_step": (ctypes.c_int, [ctypes.POINTER(MuzTttState), ctypes.c_int32, vp, vp]),
    "muz_ttt_policy_logits": (ctypes.c_int, [ctypes.POINTER(MuzTttState), vp]),
    "muz_ttt_rollout": (ctypes.c_int, [ctypes.POINTER(MuzTttState), ctypes.c_uint64, ctypes.c_uint32, vp]),
    "muz_ttt_muzero_policy": (ctypes.c_int, [ctypes.POINTER(MuzTttState), ctypes.c_int32, ctypes.c_int32,
                                             ctypes.c_double, ctypes.c_uint64, ctypes.c_int32,
                                             ctypes.POINTER(MuzTttPolicyOut)]),
    "muz_ttt_match": (ctypes.c_int, [ctypes.c_int32, ctypes.c_int32, ctypes.c_uint64, ctypes.c_int32, ctypes.c_int32,
                                     vp]),
    "muz_traj_offsets": (ctypes.c_int, [vp, ctypes.c_int32, vp, vp, vp]),
    "muz_traj_pack": (ctypes.c_int, [MuzTraj, vp, vp, ctypes.c_int32, ctypes.c_int32, ctypes.c_int32, MuzTraj, vp, vp]),
    "muz_ring_save_packed": (ctypes.c_int, [MuzRing, MuzTraj, vp, vp, ctypes.c_int32, ctypes.c_int32, ctypes.c_int32,
                                            vp, vp, vp]),
    "muz_ring_save": (ctypes.c_int, [MuzRing, MuzTraj, vp, ctypes.c_int32, ctypes.c_int32, vp, vp, vp]),
    "muz_ring_sample": (ctypes.c_int, [MuzRing, vp, vp, ctypes.c_int32, ctypes.c_int32, ctypes.c_int32, ctypes.c_int32,
                                       vp, MuzSample, vp]),
    "muz_classic_net_prepare": (ctypes.c_int, [ctypes.POINTER(MuzClassicNetW), vp]),
    "muz_classic_nets_root": (ctypes.c_int, [ctypes.POINTER(MuzClassicNetW), vp, ctypes.c_int32, vp, ctypes.c_int64,
                                             vp, vp, vp, vp]),
    "muz_classic_nets_decision": (ctypes.c_int, [ctypes.POINTER(MuzClassicNetW), vp, vp, ctypes.c_int32, vp, vp, vp,
                                                 vp, vp, vp]),
    "muz_classic_nets_chance": (ctypes.c_int, [ctypes.POINTER(MuzClassicNetW), vp, vp, ctypes.c_int32, vp, vp, vp,
                                               vp]),
    "muz_stochastic_workspace_bytes": (ctypes.c_int64, [ctypes.c_int32, ctypes.c_int32]),
    "muz_stochastic_search": (ctypes.c_int, [ctypes.POINTER(MuzClassicNetW), ctypes.POINTER(MuzStochCfg), vp, vp, vp,
                                             vp, vp, vp, vp, ctypes.c_int32, vp, ctypes.c_int64, vp, vp, vp, vp]),
    "muz_classic_selfplay_workspace_bytes": (ctypes.c_int64, [ctypes.c_int32, ctypes.c_int32,
                                                              ctypes.POINTER(MuzStochCfg)]),
    "muz_classic_selfplay": (ctypes.c_int, [ctypes.POINTER(MuzRules), ctypes.POINTER(MuzClassicNetW),
                                            ctypes.POINTER(MuzStochCfg), MuzClassicSoA, MuzTraj, MuzTrajChance,
                                            ctypes.c_int32, vp, ctypes.c_int64, ctypes.POINTER(MuzSpStats), vp]),
    "muz_classic_selfplay_stream": (ctypes.c_int, [ctypes.POINTER(MuzRules), ctypes.POINTER(MuzClassicNetW),
                                                   ctypes.POINTER(MuzStochCfg), MuzClassicSoA, MuzTraj, MuzTrajChance,
                                                   ctypes.c_int32, ctypes.c_int32, vp, ctypes.c_int64,
                                                   ctypes.POINTER(MuzSpStats), vp]),
    "muz_net_prepare": (ctypes.c_int, [ctypes.POINTER(MuzNetW), ctypes.c_void_p]),
    "muz_nets_root_scratch_bytes": (ctypes.c_int64, [ctypes.c_int32]),
    "muz_nets_root": (ctypes.c_int, [ctypes.POINTER(MuzNetW), vp, ctypes.c_int32, vp, ctypes.c_int64, vp, vp, vp,
                                     vp]),
    "muz_nets_recurrent": (ctypes.c_int, [ctypes.POINTER(MuzNetW), vp, vp, ctypes.c_int32, vp, vp, vp, vp, vp,
                                          vp]),
    "muz_search_workspace_bytes": (ctypes.c_int64, [ctypes.c_int32, ctypes.POINTER(MuzSearchCfg)]),
    "muz_gumbel_search": (ctypes.c_int, [ctypes.POINTER(MuzNetW), ctypes.POINTER(MuzSearchCfg), vp, vp, vp, vp,
                                         vp, vp, ctypes.c_int32, vp, ctypes.c_int64, vp, vp, vp, vp]),
    "muz_selfplay_workspace_bytes": (ctypes.c_int64, [ctypes.c_int32, ctypes.c_int32, ctypes.POINTER(MuzSearchCfg)]),
    "muz_detmadn_selfplay": (ctypes.c_int, [ctypes.POINTER(MuzRules), ctypes.POINTER(MuzNetW),
                                            ctypes.POINTER(MuzSearchCfg), MuzDetSoA, MuzTraj, ctypes.c_int32, vp,
                                            ctypes.c_int64, ctypes.POINTER(MuzSpStats), vp]),
    "muz_ln_fwd": (ctypes.c_int, [vp, vp, vp, vp, vp, ctypes.c_int32, ctypes.c_int32, ctypes.c_int32, vp, vp, vp, vp,
                                  vp]),
    "muz_ln_fwd_parts": (ctypes.c_int, [vp, ctypes.c_int32, vp, vp, vp, vp, ctypes.c_int32, ctypes.c_int32,
                                        ctypes.c_int32, vp, vp, vp, vp, vp]),
    "muz_ln_bwd_scratch_floats": (ctypes.c_int64, [ctypes.c_int32, ctypes.c_int32]),
    "muz_ln_bwd_rows": (ctypes.c_int, [vp, vp, vp, vp, vp, vp, ctypes.c_int32, ctypes.c_int32, ctypes.c_int32, vp, vp,
                                       vp, vp]),
    "muz_ln_bwd_rows_ld": (ctypes.c_int, [vp, ctypes.c_int32, vp, vp, vp, vp, vp, ctypes.c_int32, ctypes.c_int32,
                                          ctypes.c_int32, vp, vp, vp, vp]),
    "muz_ln_colsum": (ctypes.c_int, [vp, ctypes.c_int64, ctypes.c_int32, vp, vp, vp, vp]),
    "muz_ln_bwd": (ctypes.c_int, [vp, vp, vp, vp, vp, vp, ctypes.c_int32, ctypes.c_int32, ctypes.c_int32, vp, vp, vp,
                                  vp, vp, vp, vp]),
    "muz_film_fwd": (ctypes.c_int, [vp, ctypes.c_int32, ctypes.c_int32, vp, vp, vp, vp, vp, vp, vp, vp, vp, vp, vp,
                                    vp]),
    "muz_film_fwd_strided": (ctypes.c_int, [vp, ctypes.c_int32, ctypes.c_int32, ctypes.c_int32, ctypes.c_int32, vp,
                                            vp, vp, vp, vp, vp, vp, vp, vp, vp, vp, vp]),
    "muz_film_bwd": (ctypes.c_int, [vp, vp, vp, vp, vp, ctypes.c_int32, vp, vp]),
    "muz_ln_film_fwd": (ctypes.c_int, [vp, vp, vp, vp, vp, ctypes.c_int32, ctypes.c_int32, vp, vp, vp, vp, vp, vp]),
    "muz_ln_film_bwd_rows": (ctypes.c_int, [vp, vp, vp, vp, vp, vp, vp, ctypes.c_int32, ctypes.c_int32, vp, vp, vp,
                                            vp]),
    "muz_minmax_film_fwd": (ctypes.c_int, [vp, vp, vp, ctypes.c_int32, ctypes.c_int32, vp, vp, vp, vp, vp, vp, vp, vp,
                                           vp, vp, vp, vp, vp, vp]),
    "muz_film_minmax_bwd": (ctypes.c_int, [vp, vp, vp, vp, vp, vp, vp, ctypes.c_int32, ctypes.c_int32, vp, vp, vp,
                                           vp, vp, ctypes.c_float, ctypes.c_int32, vp, vp, vp, vp]),
    "muz_minmax_fwd": (ctypes.c_int, [vp, vp, vp, ctypes.c_int32, ctypes.c_int32, vp, vp, vp, vp, vp]),
    "muz_minmax_bwd": (ctypes.c_int, [vp, vp, vp, vp, ctypes.c_float, ctypes.c_int32, vp, vp, ctypes.c_int32,
                                      ctypes.c_int32, vp, vp]),
    "muz_im2col_fwd": (ctypes.c_int, [vp, ctypes.c_int32, ctypes.c_int32, ctypes.c_int32, ctypes.c_int32, vp, vp]),
    "muz_im2col_fwd_strided": (ctypes.c_int, [vp, ctypes.c_int32, ctypes.c_int32, ctypes.c_int32, ctypes.c_int32,
                                              ctypes.c_int64, ctypes.c_int64, ctypes.c_int64, vp, vp]),
    "muz_im2col_bwd": (ctypes.c_int, [vp, ctypes.c_int32, ctypes.c_int32, ctypes.c_int32, ctypes.c_int32, vp, vp]),
    "muz_wgrad_scratch_floats": (ctypes.c_int64, [vp, ctypes.c_int32]),
    "muz_wgrad_segment_rows": (ctypes.c_int32, []),
    "muz_wgrad_grouped": (ctypes.c_int, [vp, ctypes.c_int32, vp, ctypes.c_int64, vp]),
    "muz_colsum_grouped": (ctypes.c_int, [vp, ctypes.c_int32, vp]),
    "muz_loss_heads": (ctypes.c_int, [vp, vp]),
    "muz_heads_fwd": (ctypes.c_int, [ctypes.POINTER(MuzHeadsArgs), vp]),
    "muz_heads_bwd": (ctypes.c_int, [ctypes.POINTER(MuzHeadsArgs), vp]),
    "muz_dense_ln_fwd": (ctypes.c_int, [vp, ctypes.c_int32, ctypes.c_int32, vp, vp, ctypes.c_int32, vp, vp, vp, vp,
                                        ctypes.c_int32, ctypes.c_int32, vp, vp, vp, vp, vp]),
    "muz_transpose_grouped": (ctypes.c_int, [vp, ctypes.c_int32, vp]),
    "muz_dense_ln_bwd_scratch_floats": (ctypes.c_int64, [ctypes.c_int32, ctypes.c_int32]),
    "muz_dense_ln_bwd": (ctypes.c_int, [vp, vp, vp, vp, vp, vp, ctypes.c_int32, ctypes.c_int32, ctypes.c_int32, vp,
                                        ctypes.c_int32, vp, vp, vp, vp, vp, vp]),
    "muz_dense_ln_bwd_ld": (ctypes.c_int, [vp, ctypes.c_int32, vp, vp, vp, vp, vp, ctypes.c_int32, ctypes.c_int32,
                                           ctypes.c_int32, vp, ctypes.c_int32, vp, vp, vp, vp, vp, vp]),
    "muz_trunk_chain_pack": (ctypes.c_int, [vp, ctypes.c_int32, vp, vp, vp]),
    "muz_trunk_chain_fwd": (ctypes.c_int, [ctypes.POINTER(MuzChainArgs), vp]),
    "muz_rbstack_fwd": (ctypes.c_int, [ctypes.POINTER(MuzRbstackArgs), vp]),
    "muz_rbstack_bwd": (ctypes.c_int, [ctypes.POINTER(MuzRbstackArgs), vp]),
    "muz_trunk_chain_bwd": (ctypes.c_int, [ctypes.POINTER(MuzChainArgs), vp]),
    "muz_adamw_scratch_bytes": (ctypes.c_int64, [ctypes.c_int32, vp]),
    "muz_adamw_step": (ctypes.c_int, [vp, vp, vp, vp, vp, ctypes.c_int32, vp, vp, vp, ctypes.c_float, ctypes.c_double,
                                      ctypes.c_double, ctypes.c_float, ctypes.c_float, ctypes.c_double, ctypes.c_double,
                                      vp, ctypes.c_int32, vp]),
    "muz_adamw_table_bytes": (ctypes.c_int64, [ctypes.c_int32]),
    "muz_adamw_table_write": (ctypes.c_int, [vp, vp, vp, vp, vp, vp, ctypes.c_int32, vp]),
    "muz_adamw_step_table": (ctypes.c_int, [vp, vp, ctypes.c_int32, vp, vp, vp, ctypes.c_float, ctypes.c_double,
                                            ctypes.c_double, ctypes.c_float, ctypes.c_float, ctypes.c_double,
                                            ctypes.c_double, vp, ctypes.c_int32, vp]),
    "muz_dog_net_prepare": (ctypes.c_int, [ctypes.POINTER(MuzDogNetW), vp]),
    "muz_dog_encode": (ctypes.c_int, [ctypes.POINTER(MuzRules), MuzDogSoA, vp, ctypes.c_int32, vp]),
    "muz_dog_nets_root": (ctypes.c_int, [ctypes.POINTER(MuzDogNetW), vp, ctypes.c_int32, vp, ctypes.c_int64, vp, vp,
                                         vp, vp]),
    "muz_dog_nets_recurrent": (ctypes.c_int, [ctypes.POINTER(MuzDogNetW), vp, vp, ctypes.c_int32, vp, vp, vp, vp,
                                              vp, vp]),
    "muz_dog_search_workspace_bytes": (ctypes.c_int64, [ctypes.c_int32, ctypes.POINTER(MuzSearchCfg)]),
    "muz_dog_search_games_per_workgroup": (ctypes.c_int32, [ctypes.c_int32]),
    "muz_dog_gumbel_search": (ctypes.c_int, [ctypes.POINTER(MuzDogNetW), ctypes.POINTER(MuzSearchCfg), vp, vp, vp,
                                             vp, vp, ctypes.c_int32, vp, ctypes.c_int64, vp, vp, vp, vp]),
    "muz_detmadn_selfplay_stream": (ctypes.c_int, [ctypes.POINTER(MuzRules), ctypes.POINTER(MuzNetW),
                                                   ctypes.POINTER(MuzSearchCfg), MuzDetSoA, MuzTraj, ctypes.c_int32,
                                                   ctypes.c_int32, vp, ctypes.c_int64, ctypes.POINTER(MuzSpStats),
                                                   vp]),
}

_lib = None


class MuzError(RuntimeError):
    pass


def load():
    """Load libmuz.so (raises if it was not built -- there is no fallback)."""
    global _lib
    if _lib is not None:
        return _lib
    if os.environ.get("MUZ_LIB"):       # never silent: a diagnostic build gives different timings
        import sys
        print(f"libmuz: MUZ_LIB selects {LIB_PATH} instead of the in-tree libmuz.so", file=sys.stderr)
    if not os.path.exists(LIB_PATH):
        raise MuzError(f"{LIB_PATH} is missing: build it with `python -c 'import __graft_entry__ as g; g.build()'`")
    # torch must own the HIP runtime first so both share one libamdhip64.so.7 instance.
    import torch  # noqa: F401
    lib = ctypes.CDLL(LIB_PATH)
    for name, (res, args) in SIGNATURES.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    _lib = lib
    return lib


def check(rc: int, what: str = ""):
    if rc != MUZ_OK:
        msg = load().muz_error_string(rc).decode()
        raise MuzError(f"{what} failed: {msg} (code {rc})")


def stream_ptr(stream=None):
    import torch
    s = stream if stream is not None else torch.cuda.current_stream()
    return ctypes.c_void_p(s.cuda_stream)


def ptr(t):
    return ctypes.c_void_p(0 if t is None else t.data_ptr())


def nbytes(t):
    return t.numel() * t.element_size()
