/*
 * blokus_engine.h — C-ABI of the MI355X-native Blokus engine (libblokus_hip.so).
 *
 * This is the drop-in boundary for the reference's hot path. The reference
 * reaches its rules engine (the un-vendored `colosseumrl.envs.blokus`, setup.py:11) through
 * `ColosseumBlokusGameWrapper` (blokus_rl/colossumrl/blokus_wrapper.py:21) and its search through
 * `MCTS` (blokus_rl/alphazero/mcts.py:7). Every entry point below names the reference interface
 * it replaces. The Python mirror of those classes (blokus_rl_amd/) binds this header via ctypes;
 * INTEGRATION.md shows the binding.
 *
 * Conventions
 *   - Plain C types only. Device buffers are raw device pointers (e.g. torch `data_ptr()`),
 *     caller-owned, and every launch takes a `stream` (a hipStream_t passed as void*; NULL =
 *     the null stream). No call synchronises unless its comment says so.
 *   - Return 0 on success, a negative BK_E* code on failure; bk_last_error() returns text.
 *   - One context per stream; a context is not thread-safe.
 *   - States are values: no call mutates an input state (blokus_wrapper.py:89-106 semantics).
 */
#ifndef BLOKUS_ENGINE_H
#define BLOKUS_ENGINE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---------------------------------------------------------------- error codes */
#define BK_OK 0
#define BK_EINVAL -1    /* bad argument (null pointer, size, preset)            */
#define BK_EHIP -2      /* a HIP runtime call failed                             */
#define BK_EILLEGAL -3  /* an action is not legal in its state (next_state)     */
#define BK_ECAPACITY -4 /* an MCTS pool/table ran out of room                    */
#define BK_ENOMEM -5    /* the requested device allocation exceeds free memory  */

/* ---------------------------------------------------------------- packed state
 * One game state = 384 bytes (6 x 64 B), 64-B aligned in arrays. Byte layout:
 *   [  0,320) uint32 occ[4][20]   occupancy bitboard per colour; row r, bit c = cell (r,c).
 *                                 Colours 0..P-1 = reference colours 1..P
 *                                 (blokus_wrapper.py:259 colour map).
 *   [320,336) uint32 pieces[4]    bit i set = piece i still unused by that colour.
 *   [336,344) uint64 hash         64-bit hash of the board contents only (occ), the analogue
 *                                 of hash(board_contents.tobytes()) (blokus_wrapper.py:208-218).
 *   [344,348) int32  to_move      player to move (reference `current_player`).
 *   [348,352) int32  ply          placements made so far.
 *   [352,356) uint32 flags        bit0 = game over (nobody can move);
 *                                 bits 4..7 = player known to have no legal move (cache).
 *   [356,384) reserved, zero.
 */
#define BK_STATE_BYTES 384
#define BK_MAX_N 20
#define BK_MAX_P 4

typedef struct bk_ctx bk_ctx;
typedef struct bk_mcts bk_mcts;

const char* bk_last_error(void);
int bk_version(void);
int bk_state_bytes(void);

/* ---------------------------------------------------------------- context / presets
 * board_size N (5..20), num_players P (2 or 4), max_piece_cells (1..5).
 * Presets used by the reference: (20,4,5) -> 30433 actions (docs/README.md:128);
 * (7,2,4) -> 919 actions (docs/README.md:51); (7,2,5) -> 2522 (the 7x7 recordings).
 * device < 0 creates a host-only context (tables only; every device call then fails).
 * Replaces: BlokusEnvironment() + _set_all_possible_moves (blokus_wrapper.py:42, :281-324). */
int bk_ctx_create(int board_size, int num_players, int max_piece_cells, int device, bk_ctx** out);
int bk_ctx_destroy(bk_ctx* ctx);
/* get_action_size (blokus_wrapper.py:59-64). */
int bk_action_size(const bk_ctx* ctx);
/* Number of u64 words of one legal-move bitmask = ceil(A/64). */
int bk_mask_words(const bk_ctx* ctx);
/* Host copy of the action table: out[4*id + {0,1,2,3}] = {piece, orientation, row, col} of
 * the placement's bounding-box origin. Canonical id order = (piece, orientation, row, col).
 * Replaces the action-string <-> id dicts (blokus_wrapper.py:37-38, :313-318). */
int bk_action_table(const bk_ctx* ctx, int32_t* out);
/* Host copy of the placement cells: out[5*id + k] = row*N + col of cell k, -1 padded. */
int bk_action_cells(const bk_ctx* ctx, int16_t* out);
/* Piece count in this preset (21 at max_piece_cells 5, 9 at 4). */
int bk_num_pieces(const bk_ctx* ctx);

/* ---------------------------------------------------------------- batched env (device)
 * get_init_board (blokus_wrapper.py:80-87): B fresh states, player 0 to move. */
int bk_init_states(bk_ctx* ctx, void* states, int B, void* stream);

/* get_valid_moves (blokus_wrapper.py:108-132) for B states. players[b] = player whose moves
 * are listed, or -1 (or players == NULL) for the state's to_move (the wrapper's -1 convention,
 * :119-121). mask_words: [B][bk_mask_words] u64, bit id set = legal. counts: [B] int32 (may be
 * NULL). Legality = cells empty, no own-colour edge contact, >=1 own-colour corner contact
 * (own start corner on the colour's first placement), piece unused. */
int bk_legal_mask(bk_ctx* ctx, const void* states, const int32_t* players, int B,
                  uint64_t* mask_words, int32_t* counts, void* stream);

/* get_next_state (blokus_wrapper.py:89-106) for B states: place actions[b] for the state's
 * to_move, retire the piece, then pass the turn to the next player in cyclic order who has a
 * legal move (skip rule); nobody -> game over. states_out may alias nothing in states_in.
 * next_players: [B] int32 (may be NULL). status: [B] int32 (may be NULL): 0 ok, 1 illegal
 * action (state copied unchanged). actions[b] < 0 -> state copied unchanged (status 0). */
int bk_next_state(bk_ctx* ctx, const void* states_in, const int32_t* actions, int B,
                  void* states_out, int32_t* next_players, int32_t* status, void* stream);

/* get_game_ended (blokus_wrapper.py:164-186): ended[b] = 1 when nobody can move; then
 * scores[b][P] = -1 for losers, 3 for a sole winner, 1 for each tied winner (winner = most
 * squares placed); 0-filled when not ended. */
int bk_game_ended(bk_ctx* ctx, const void* states, int B, int32_t* ended, double* scores,
                  void* stream);

/* Board.canonical_board via get_observation (blokus_wrapper.py:134-146): obs[B][2P][N][N] f32;
 * planes 0..P-1 = colour occupancy (absolute orientation), plane P+to_move = all ones. */
int bk_observe(bk_ctx* ctx, const void* states, int B, float* obs, void* stream);

/* Squares placed per colour: out[B][P] int32 (scoring input of get_winners). */
int bk_square_counts(bk_ctx* ctx, const void* states, int B, int32_t* out, void* stream);

/* Compact legal ids: ids[b][0..K) ascending (the np.where(mask) order of mcts.py:64),
 * counts[b] = K; rows are `cap` ids wide (K > cap -> BK_ECAPACITY flagged in counts as -K). */
int bk_legal_ids(bk_ctx* ctx, const void* states, const int32_t* players, int B, int32_t* ids,
                 int cap, int32_t* counts, void* stream);

/* ---------------------------------------------------------------- batched MCTS (device)
 * T independent search trees (one per game), one simulation in flight per tree, which keeps
 * each tree's sequence of simulations identical to MCTS.simulate (mcts.py:13-71). A tree is a
 * transposition table keyed by the board hash (mcts.py:37-39) with SoA child statistics
 * {id, N, Q (f64), P (f32)}; it persists across moves of one game (trainer.py:95).
 *   node_cap  : nodes per tree (hash table sized to 2x that, power of two)
 *   child_cap : total child slots, split evenly into one region per tree */
int bk_mcts_create(bk_ctx* ctx, int trees, int node_cap, int64_t child_cap, bk_mcts** out);
int bk_mcts_destroy(bk_mcts* m);
/* Clear the trees whose flag is non-zero (reset_flags: [T] int32 device, NULL = all):
 * MCTSPlayer.reset / a new MCTS(game, nn) per episode (mcts_player.py:24-25, trainer.py:95). */
int bk_mcts_reset(bk_mcts* m, const int32_t* reset_flags, void* stream);

/* One selection pass (the descent half of simulate, mcts.py:37-50 and :58-65): for every tree
 * with active[t] != 0 descend from roots[t] by argmax(Q + cpuct*P*sqrt(sum N + 1e-6)/(1+N))
 * (first max; cpuct only at the root, as mcts.py:50 passes none further) until a board not in
 * the table or a terminal board. Outputs per tree:
 *   leaf_status[t]: 0 inactive, 1 needs NN evaluation, 2 terminal (value = one-hot scores)
 *   obs[t]: the leaf observation [2P][N][N] f32 (written for status 1) — the NN input batch
 *   leaf_mask: [T][mask_words] legal bits of the leaf (status 1), for the masked softmax; may be
 *   null (the engine keeps its own copy for the expansion). */
int bk_mcts_select(bk_mcts* m, const void* roots, const int32_t* active, double cpuct,
                   int32_t* leaf_status, float* obs, uint64_t* leaf_mask, void* stream);
/* The same with the root's exploration term under the square root given: mcts.py:43 adds
 * (1e-6 if epsilon_fix else 0) to N.sum() at the root only (the recursive call of mcts.py:50
 * passes the default epsilon_fix=True, so every deeper level uses 1e-6). root_eps = 1e-6 is
 * bk_mcts_select; MCTS.simulate(..., epsilon_fix=False) passes 0. */
int bk_mcts_select_eps(bk_mcts* m, const void* roots, const int32_t* active, double cpuct, double root_eps,
                       int32_t* leaf_status, float* obs, uint64_t* leaf_mask, void* stream);

/* Expansion + backup (mcts.py:50-56 and :63-70): for status-1 leaves create the node with
 * P = exp(log_softmax(logp[t][legal ids])) (neural_network.py:159-173) and back up
 * values[t][P]; for status-2 leaves back up the terminal scores. logp: [T][A] f32 (the net's
 * log-softmax output or raw logits — the softmax over the legal ids is shift-invariant; rows of
 * inactive/terminal trees ignored); values: [T][P] f32.
 * prior_mode 0: dense logp as above; 1 (test hook): logp[t][id] already holds the prior P at
 * the legal ids, no softmax — lets a test feed the reference MCTS and this engine identical
 * priors; 2: the sparse logits of bk_mcts_leaf_logits (logp may be NULL). */
int bk_mcts_expand_backup(bk_mcts* m, const float* logp, const float* values, int prior_mode,
                          void* stream);

/* The policy head's last Linear restricted to each leaf's legal ids (prior_mode 2 input):
 * for every tree whose last select pass stopped at a leaf needing evaluation, logit_j =
 * W[id_j] . feat[t] + bias[id_j] over the leaf's K legal ids (ascending), kept inside the
 * search state (K <= 2048, else error bit 32). feat [T][ldf] f32 (the policy features, F of
 * them), W [A][F], bias [A] (policy_out of models/blokus_nnet.py:147, the same parameters the
 * dense head multiplies). Replaces the [T, A] GEMM + gather: only the K ~ 200 logits of the
 * legal ids are computed. */
int bk_mcts_leaf_logits(bk_mcts* m, const float* feat, int64_t ldf, int F, const float* W, const float* bias,
                        void* stream);

/* The search half of a simulation and the descent of the next, in one launch (k_leaf_step, one
 * workgroup per tree): bk_mcts_leaf_logits(feat, ldf, F, W, bias) -> bk_mcts_expand_backup(NULL,
 * values, 2) -> (do_select) bk_mcts_select(roots, active, cpuct, leaf_status, obs, leaf_mask),
 * the same trees bitwise, without the grid-wide step between the three. Replaces, inside the
 * simulation loop (trainer.py:104-105), the end of one MCTS.simulate (mcts.py:60-70, the priors
 * of predict, neural_network.py:92-110) and the descent of the next (mcts.py:37-50). */
int bk_mcts_leaf_step(bk_mcts* m, const float* feat, int64_t ldf, int F, const float* W, const float* bias,
                      const float* values, int do_select, const void* roots, const int32_t* active, double cpuct,
                      int32_t* leaf_status, float* obs, uint64_t* leaf_mask, void* stream);

/* get_distribution (mcts.py:73-99) at the root of every active tree: ids[t][0..K) and
 * pi[t][0..K) (f64) in child order, K in counts[t]; temperature 0 -> one-hot argmax N
 * (first max); all-zero N -> uniform. Rows are `cap` wide. Root must be expanded. */
int bk_mcts_root_policy(bk_mcts* m, const void* roots, const int32_t* active, double temperature,
                        int32_t* ids, double* pi, int cap, int32_t* counts, void* stream);

/* Root child statistics (for tests / players): n[t][cap] u32, q[t][cap] f64, p[t][cap] f32. */
int bk_mcts_root_stats(bk_mcts* m, const void* roots, const int32_t* active, int32_t* ids,
                       uint32_t* n, double* q, float* p, int cap, int32_t* counts, void* stream);

/* Leaf of the last select pass, per tree: leaf_states [T][384] (device), depths [T] int32. */
int bk_mcts_leaf_info(bk_mcts* m, void* leaf_states, int32_t* depths, void* stream);

/* Engine counters (host copy, synchronises the stream): out[0] nodes used (all trees),
 * out[1] children used, out[2] selection levels descended (cumulative), out[3] leaves
 * expanded, out[4] terminal leaves, out[5] error flags (bit0 child pool full, bit1 table full,
 * bit2 depth, bit3 illegal child, bit4 root missing), out[6] children scanned by selection
 * (sum of K over descended nodes), out[7] children created by expansion. */
int bk_mcts_counters(bk_mcts* m, int64_t* out, void* stream);

/* The self-play ply's tail after the search, per game g < G (trainer.py:108-137; one launch each
 * instead of the per-op tensor code). bk_ply_policy: from bk_mcts_root_policy's ids/pi/counts
 * rows (`cap` wide), on a game's first ply (first_ply[g] != 0) pi = (1 - w) pi + w Dir(alpha) over
 * its counts[g] legal ids (trainer.py:110-116, float64), pi32 = float32(pi) (trainer.py:124), the
 * action = ids[g][i] with i drawn from pi32 (np.random.choice, trainer.py:125) or -1 when the game
 * is inactive or has no legal id (counts <= 0); record fields ids16 (int16 ids, 0 past K), pi32
 * (0 past K), act_mask (1 = the game moved), player (the mover). Random numbers are counter-based
 * in (seed, ply, g): one call per ply with a new `ply` value. 0 < cap <= 4096.
 * bk_ply_finish (one workgroup): games with active && ended store z_table[game_id] = scores
 * (float32, trainer.py:134-135) and z_known = 1, get reset_flags = 1 (for bk_mcts_reset: a new
 * tree per episode, trainer.py:95) and count into fin_count; continuous != 0 restarts them from
 * init_state (one state) with ids *next_gid + (finished games before g), advancing *next_gid;
 * otherwise active[g] = 0. first_ply = (first_ply && !act_mask) || restarted; sims_count +=
 * num_sims x (games that moved); cap_overflow = 1 if an active game had counts < 0. roots_out
 * (a different buffer than roots) receives the next roots, game_id_out the next ids. */
int bk_ply_policy(const int32_t* ids, const double* pi, const int32_t* counts, const int32_t* active,
                  const uint8_t* first_ply, int G, int cap, double dirichlet_weight, double dirichlet_alpha,
                  uint64_t seed, uint64_t ply, const void* roots, int32_t* action, int16_t* ids16, float* pi32,
                  uint8_t* act_mask, int32_t* player, void* stream);
int bk_ply_finish(int G, int P, const int32_t* ended, const double* scores, const int32_t* counts,
                  const uint8_t* act_mask, const int64_t* game_id, const void* roots, const void* init_state,
                  int continuous, int num_sims, int32_t* active, uint8_t* first_ply, int32_t* reset_flags,
                  int64_t* game_id_out, void* roots_out, float* z_table, uint8_t* z_known, int64_t zcap,
                  int64_t* next_gid, int64_t* fin_count, int64_t* sims_count, int32_t* cap_overflow, void* stream);

/* ---------------------------------------------------------------- config 5: PPO vector env
 * The blokus_gym `blokus-simple-v0` env as the PPO trainer drives it (ppo/trainer.py:128-175,
 * :380-386): 2-player preset, the agent is colour 0 against a built-in uniform-random opponent
 * (colour 1), reward +1 / 0 / -1 at the episode's end, auto-reset. E envs, states [E][384],
 * rng [E] u64 per-env counters, obs [E][N*N] u8 (0 empty, 1 agent, 2 opponent), mask
 * [E][mask_words] (the agent's legal ids = `ai_possible_indexes`), reward [E] f32, done [E].
 * bk_vec_reset: fresh episodes, rng[e] = seeds[e] (seeds NULL keeps rng).
 * bk_vec_step: actions[e] = the agent's id (< 0, or actions NULL: a uniformly random legal id
 * drawn in-kernel — the benchmark's policy stand-in); an illegal id ends the episode as a loss. */
int bk_vec_reset(bk_ctx* ctx, void* states, uint64_t* rng, const uint64_t* seeds, int E, uint8_t* obs,
                 uint64_t* mask, void* stream);
int bk_vec_step(bk_ctx* ctx, void* states, uint64_t* rng, const int32_t* actions, int E, uint8_t* obs,
                uint64_t* mask, float* reward, int32_t* done, void* stream);
/* bk_vec_policy: the agent's moves drawn from its policy, as the PPO rollout draws them
 * (ppo/trainer.py:144-155 -> get_action_and_value, ppo/agent.py:148-156: the actor's logits
 * through FilterLegalMoves, :27-42, then Categorical(logits).sample() / .log_prob()), replacing
 * the [E][A] filter + softmax + multinomial of that call. logits [E][A] f32 (the actor's raw
 * output), mask [E][mask_words] (the agent's legal ids, as bk_vec_reset / bk_vec_step leave
 * them). Candidates: the legal ids, minus those whose logit is exactly 0 when zero_masked != 0
 * (the reference filter's quirk); with none, every id in [0, A) at -1e9 (uniform, as the
 * reference's all -1e9 row). actions[e] is drawn from the softmax over the candidates by an
 * inverse CDF on the env's splitmix64 stream (one draw; rng[e] advanced), logp[e] =
 * logits[e][a] - logsumexp (Categorical.log_prob). Feed actions to bk_vec_step. 2-player 7x7
 * presets (919 / 2522 ids). */
int bk_vec_policy(bk_ctx* ctx, const float* logits, const uint64_t* mask, uint64_t* rng, int E, int zero_masked,
                  int32_t* actions, float* logp, void* stream);
/* bk_vec_step_policy: one rollout step in one launch — the agent's id drawn from its policy
 * logits exactly as bk_vec_policy draws it (same arithmetic, the legal mask taken from the step's
 * own legality pass instead of HBM), written to actions / logp, then bk_vec_step with that id:
 * the two launches' results bit for bit. The 2-player 7x7 presets. */
int bk_vec_step_policy(bk_ctx* ctx, void* states, uint64_t* rng, const float* logits, int zero_masked, int E,
                       uint8_t* obs, uint64_t* mask, float* reward, int32_t* done, int32_t* actions, float* logp,
                       void* stream);

/* ---------------------------------------------------------------- learner
 * Packed replay row (blokus_rl_amd/replay.py), fixed stride bk_replay_stride(cap), 16-B aligned:
 *   state 384 B | K int32 | player int32 | z f32[4] | ids int16[cap] (ascending legal ids, -1
 *   padded) | pi f32[cap].  cap is a multiple of 64. */
size_t bk_replay_stride(int cap);

/* The training-batch loader: replaces AlphaZeroDataset.__getitem__ + collate_dataset_fn
 * (alphazero/dataset.py:38-54) and train_step's host->device copy (neural_network.py:64).
 * For b < B, row index[b] of `rows` -> obs[b][2P][N][N] f32 (the get_observation planes),
 * ids[b][cap], pi[b][cap], k[b], z[b][P]; states[b][384] too when states != NULL. */
int bk_replay_batch(bk_ctx* ctx, const void* rows, int cap, const int64_t* index, int B, float* obs,
                    int16_t* ids, float* pi, int32_t* k, float* z, void* states, void* stream);

/* Policy term of BlokusNNetWrapper.compute_loss (neural_network.py:138-157, with
 * get_valid_dist(log_softmax=True), :159-173) over sparse search policies: for each row b,
 * loss[b] = -sum_{j<k[b]} pi[b][j] * log_softmax(x[b][ids[b][0..k[b])])_j and lse[b] = the
 * log-partition of the row's legal logits. x is [B][ldx] f32 (the net's policy output). */
int bk_policy_loss(const float* x, int64_t ldx, const int16_t* ids, const float* pi, const int32_t* k, int cap,
                   int B, float* loss, float* lse, void* stream);

/* Its gradient: grad[b][ids[b][j]] = s * (S_b * exp(x[b][ids[b][j]] - lse[b]) - pi[b][j]),
 * S_b = sum_j pi[b][j], s = scale * (*gscale) (gscale: a device f32, the upstream gradient, or
 * NULL for 1); entries at other ids are left untouched (the caller zero-fills). */
int bk_policy_loss_grad(const float* x, int64_t ldx, const int16_t* ids, const float* pi, const int32_t* k,
                        int cap, int B, const float* lse, float scale, const float* gscale, float* grad,
                        int64_t ldg, void* stream);

/* The learner's 3x3 convolutions 64 -> 64 (stride 1, zero padding 1; the residual tower of
 * models/blokus_nnet.py:103-112 as neural_network.py:52-85 trains it) on split-f16 MFMA products
 * with fp32-class accuracy (trainconv.hip: the leaf net's x3 arithmetic, one launch per conv):
 * y[b][p][o] = sum_{tap, c} W[o][c][tap] x[b][p + tap][c] (+ bias[o]), x and y NHWC
 * [B][N][N][64] f32, N = 20. The forward pass uses W = the layer's weight; the input gradient
 * uses the same call on dy with W[o][c][tap] = weight[c][o][8 - tap] (bk_conv_x3_pack flip = 1).
 * wsplit (bk_conv_x3_weight_bytes() bytes) and inv [64] come from bk_conv_x3_pack on the device
 * (weight [64][64][3][3] f32, PyTorch's Conv2d layout). Replaces the fp32 convolution calls
 * (MIOpen) of the training step; bias may be NULL. */
int bk_conv_x3_weight_bytes(void);
/* The weight gradient of the same conv on split-f16 MFMA products: dw[o][c][ky][kx] (PyTorch's
 * layout, f32) = sum over b and pixels p of dy[b][p][o] * x[b][p + (ky - 1, kx - 1)][c] (zero
 * padding); x, dy NHWC [B][N][N][64] f32, N = 20; workspace: bk_conv_x3_wgrad_workspace_floats(B)
 * floats (per-workgroup partial sums, added in a fixed order: deterministic). Replaces the
 * fp32 weight-gradient convolution (MIOpen) of the training step. */
int bk_conv_x3_wgrad_workspace_floats(int B);
int bk_conv_x3_wgrad(const float* x, const float* dy, int B, int N, float* workspace, float* dw, void* stream);
int bk_conv_x3_pack(const float* w, int flip, void* wsplit, float* inv, void* stream);
int bk_conv_x3(const float* x, int B, int N, const void* wsplit, const float* inv, const float* bias, float* y,
               void* stream);

/* The learner's train-mode batch norm of a 64-channel NHWC activation x [M][64] f32 (M = batch
 * x pixels; nn.BatchNorm2d(64) of models/blokus_nnet.py:99-112 in neural_network.py:52-85's
 * train_step): batch mean / biased variance summed in fp64 (one read of x), y = (x - mean)
 * gamma / sqrt(var + eps) + beta, running_mean / running_var updated in place as PyTorch does
 * (momentum, unbiased variance; either may be NULL). stats [256] f32 receives mean, invstd,
 * scale, shift (the backward's input); workspace: bk_bn_workspace_doubles() doubles. The
 * backward: dx = dL/dx, dgamma, dbeta (may be NULL) from dy and x (one read of both for the
 * sums, one pass for dx); coef [192] f32 scratch. gamma / beta may be NULL (1 / 0). */
int bk_bn_workspace_doubles(void);
int bk_bn_forward(const float* x, int64_t M, const float* gamma, const float* beta, float* running_mean,
                  float* running_var, float momentum, float eps, double* workspace, float* stats, float* y,
                  void* stream);
int bk_bn_backward(const float* dy, const float* x, int64_t M, const float* gamma, const float* stats, double* workspace,
                   float* coef, float* dgamma, float* dbeta, float* dx, void* stream);
/* The same with the block's ReLU fused (models/blokus_nnet.py:103-112 / :137: relu(bn(conv(x))))
 * and the feeding conv's bias gradient: bk_bn_forward_ex with relu != 0 writes y = max(bn(x), 0);
 * bk_bn_backward_ex with relu != 0 takes dy = the ReLU output's gradient (masked where the
 * forward's bn(x) was not positive, recomputed from x and stats: no extra read); dsum (may be
 * NULL) receives the per-channel sum of dx over the M rows (= the bias gradient of the conv whose
 * output x is), summed in fp64 in a fixed order; workspace2: bk_bn_workspace2_doubles() doubles. */
int bk_bn_workspace2_doubles(void);
int bk_bn_forward_ex(const float* x, int64_t M, const float* gamma, const float* beta, float* running_mean,
                     float* running_var, float momentum, float eps, double* workspace, float* stats, float* y, int relu,
                     void* stream);
int bk_bn_backward_ex(const float* dy, const float* x, int64_t M, const float* gamma, const float* stats,
                      double* workspace, float* coef, float* dgamma, float* dbeta, float* dx, int relu, float* dsum,
                      double* workspace2, void* stream);

/* The learner's policy Linear (models/blokus_nnet.py:144-146 policy_out, F = 2N^2 -> A) only where
 * compute_loss reads it (neural_network.py:138-157: the log-softmax over each row's legal ids),
 * replacing the three dense fp32 GEMMs of its forward and backward (trainfc.hip). pf [B][F] f32,
 * W [A][F] f32 (nn.Linear's layout), bias [A], ids [B][cap] int16 (the replay's legal ids, read as
 * unsigned, distinct within a row), k [B]; F % 4 == 0, F <= 1024; an id outside [0, A) is ignored
 * (its logit is 0, it enters no gradient); sums in a fixed order (deterministic).
 * bk_sparse_linear_fwd: xs[b][j] = bias[ids[b][j]] + pf[b] . W[ids[b][j]] for j < k[b], 0 beyond.
 * bk_sparse_linear_dx:  dpf[b] = sum_{j<k[b]} g[b][j] W[ids[b][j]]   (g [B][cap]).
 * bk_sparse_linear_index: the (id -> pairs) index for dw, in two calls: start NULL (count [A]
 *   zeroed by the caller): per-id counts; then start [A + 1] = the exclusive scan of count and
 *   cursor [A] zeroed: pairs [B cap] = the pair indices b cap + j grouped by id.
 * bk_sparse_linear_dw:  dW[a] = sum over the rows b holding id a of g[b][j] pf[b] (ascending b),
 *   db[a] likewise; every row written (zero where no row holds a); B <= 4096. */
int bk_sparse_linear_fwd(const float* pf, int B, int F, const float* W, const float* bias, int A, const int16_t* ids,
                         const int32_t* k, int cap, float* xs, void* stream);
int bk_sparse_linear_dx(const float* g, int B, int F, const float* W, int A, const int16_t* ids, const int32_t* k,
                        int cap, float* dpf, void* stream);
int bk_sparse_linear_index(const int16_t* ids, const int32_t* k, int cap, int B, int A, int32_t* count,
                           int32_t* start, int32_t* cursor, int32_t* pairs, void* stream);
int bk_sparse_linear_dw(const float* g, const float* pf, int B, int F, int cap, int A, const int32_t* start,
                        const int32_t* pairs, float* dW, float* db, void* stream);

/* ---------------------------------------------------------------- PPO
 * PPOTrainer._compute_gae (ppo/trainer.py:177-211) + returns = advantages + values (:83) for a
 * rollout of T steps x E envs ([T][E] f32, row t = step t): float32, the reference's operation
 * order; gamma_lambda = (float)(gamma * gae_lambda) computed in double, as Python does. */
int bk_ppo_gae(int T, int E, const float* rewards, const float* values, const float* dones, const float* next_value,
               const float* next_done, float gamma, float gamma_lambda, float* advantages, float* returns,
               void* stream);

/* FilterLegalMoves (ppo/agent.py:27-42) from legal-move bitmasks: out = x * mask, entries equal
 * to 0 (illegal, or a legal logit of exactly 0, as in the reference) set to -1e9. x, out [E][A]. */
int bk_filter_legal(const float* x, int E, int A, const uint64_t* mask, int mask_words, float* out, void* stream);

/* ---------------------------------------------------------------- leaf-evaluator epilogue
 * The conv epilogues of the inference ResNet (models/blokus_nnet.py:135-151, BN folded):
 * in place on x[n] (NHWC, C channels innermost): x = act(x + bias[c] (+ residual)), act = ReLU
 * when relu != 0. residual may be NULL. */
int bk_bias_act(float* x, int64_t n, int C, const float* bias, const float* residual, int relu, void* stream);

/* 3x3 convolution, stride 1, zero padding 1, 64 output channels, with the fused epilogue
 * y = act(conv(x) + bias (+ residual)), f32. Layouts: cin 64 input, y and residual are NHWC
 * [B][N][N][64]; cin 4 or 8 input is planar [B][cin][N][N] (the observation). wpacked: the 9*cin*64 weights in the kernel's MFMA operand order
 * (blokus_rl_amd/nets.py pack_conv3x3 documents it; cin 64 appends the Winograd F(2x2,3x3)
 * transformed weights, used at even N); bk_conv3x3_packed_floats(cin) = its length.
 * BK_CONV_DIRECT=1 in the environment forces the direct form for every shape.
 * Replaces conv + BN (folded) + ReLU (+ residual add) of blokus_nnet.py:135-146. */
int bk_conv3x3_packed_floats(int cin);
/* Which form bk_conv3x3 runs for (N, cin): 1 = Winograd F(2x2,3x3) (cin 64, even N), 0 = direct. */
int bk_conv3x3_form(int N, int cin);
/* The ResNet heads (blokus_nnet.py:146-150, BN folded) from the tower output x [B][NN][64] NHWC:
 * pf[B][2*NN] = relu(1x1 conv 64->2 + bp) flattened channel-major (the policy Linear's input),
 * v[B][P] = tanh(W2 relu(W1 relu(1x1 conv 64->1 + bv) + b1) + b2); wp [2][64], wv [64],
 * w1t [NN][64] (value_fc1.weight transposed), w2 [P][64] (row-major). */
int bk_resnet_heads(const float* x, int B, int NN, const float* wp, const float* bp, const float* wv, const float* bv,
                    const float* w1t, const float* b1, const float* w2, const float* b2, int P, float* pf,
                    float* vout, void* stream);
int bk_conv3x3(const float* x, int B, int N, int cin, const float* wpacked, const float* bias, const float* residual,
               int relu, float* y, void* stream);
/* The whole residual tower of the inference ResNet (blokus_nnet.py:140-141 with the block
 * structure of :103-112, BN folded) in one launch, one workgroup per board: nlayers = 2 x blocks
 * 3x3 convs 64->64, ReLU after each block's first conv, out = relu(x0 + tower(x0)). x0, hA, hB, out
 * are NHWC [B][N][N][64] (hA, hB scratch); u2all [nlayers][bk_tower_u_floats()] holds each layer's
 * Winograd U in the form-2 register order (nets.py pack_tower), biasall [nlayers][64].
 * Supported N: 14, 20 (bk_tower_supported). Same arithmetic as nlayers bk_conv3x3 calls. */
int bk_tower_u_floats(void);
int bk_tower_supported(int N);
int bk_resnet_tower(const float* x0, int B, int N, int nlayers, const float* u2all, const float* biasall, float* hA,
                    float* hB, float* out, void* stream);
/* The tower followed by the heads in the same launch (blokus_nnet.py:140-150): the last conv's
 * epilogue takes the 1x1 convs, then the value MLP runs per board; pf, vout, and the head weights
 * as bk_resnet_heads. out may be NULL (the tower output is then not written). */
int bk_resnet_tower_heads(const float* x0, int B, int N, int nlayers, const float* u2all, const float* biasall,
                          float* hA, float* hB, float* out, const float* wp, const float* bp, const float* wv,
                          const float* bv, const float* w1t, const float* b1, const float* w2, const float* b2, int P,
                          float* pf, float* vout, void* stream);
/* The whole leaf ResNet body in one launch: the stem conv (8 observation planes -> 64, + bias,
 * ReLU; blokus_nnet.py:137) from the planar observation obs [B][8][N][N] into x0 (written), then
 * bk_resnet_tower_heads. wstem: bk_stem_tower_u_floats() floats in the kernel's MFMA order
 * (nets.py pack_stem_tower), bstem [64]. */
int bk_stem_tower_u_floats(void);
int bk_resnet_stem_tower_heads(const float* obs, int B, int N, int cin, const float* wstem, const float* bstem,
                               int nlayers, const float* u2all, const float* biasall, float* x0, float* hA, float* hB,
                               float* out, const float* wp, const float* bp, const float* wv, const float* bv,
                               const float* w1t, const float* b1, const float* w2, const float* b2, int P, float* pf,
                               float* vout, void* stream);

/* The whole leaf ResNet body (models/blokus_nnet.py:135-150, eval-mode BN folded; the net the
 * reference's BlokusNNetWrapper.predict runs per leaf, neural_network.py:92-110) in one launch,
 * one workgroup per board, on the f16 matrix cores with fp32-class accuracy: every fp32 operand
 * is scaled by a power of two and split into two f16 halves, products taken as hi*hi + lo*hi +
 * hi*lo with f32 accumulation (leafnet.hip). obs [B][8][N][N] f32 (planar observation) -> policy
 * features pf [B][2NN] (relu(policy 1x1 conv), channel-major) and values vout [B][P]
 * (tanh(value MLP)); out (may be NULL): the tower output [B][N][N][64] f32. wstem / wtower:
 * split weights in the kernel's fragment order (nets.py pack_x3; bk_leafnet_x3_weight_bytes(8)
 * and nlayers x bk_leafnet_x3_weight_bytes(64) bytes), sstem [64] / stower [nlayers][64] the
 * inverse weight scales, bstem [64] / btower [nlayers][64] the biases, bounds [nlayers + 1][2]
 * per conv (stem first) (A, B) with |conv(x) + b| <= A max|x| + B (the output scale); head weights
 * as bk_resnet_heads. N = 14 or 20 (bk_leafnet_x3_supported), cin = 8, nlayers >= 1. */
int bk_leafnet_x3_weight_bytes(int cin);
int bk_leafnet_x3_supported(int N);
int bk_leafnet_x3(const float* obs, int B, int N, int cin, const void* wstem, const float* sstem, const float* bstem,
                  int nlayers, const void* wtower, const float* stower, const float* btower, const float* bounds,
                  const float* wp, const float* bp, const float* wv, const float* bv, const float* w1t, const float* b1,
                  const float* w2, const float* b2, int P, float* pf, float* vout, float* out, void* stream);

/* The same network and outputs as bk_leafnet_x3 with the residual tower as Winograd F(2x2,3x3)
 * convolutions on the same split-f16 products (leafnet_w3.hip: 16 products per 2x2 output tile
 * instead of 36). utower: nlayers x bk_leafnet_w3_weight_bytes() bytes of split U = G g G^T per
 * conv in the kernel's fragment order (nets.py pack_w3), stower [nlayers][64] its inverse scales;
 * the stem operands, btower, bounds and the heads as bk_leafnet_x3. x0ws: a workspace of
 * B x N x N x 64 floats (the stem output, kept for the tower's residual). N = 20
 * (bk_leafnet_w3_supported), cin = 8, nlayers >= 1. */
int bk_leafnet_w3_weight_bytes(void);
int bk_leafnet_w3_supported(int N);
int bk_leafnet_w3(const float* obs, int B, int N, int cin, const void* wstem, const float* sstem, const float* bstem,
                  int nlayers, const void* utower, const float* stower, const float* btower, const float* bounds,
                  const float* wp, const float* bp, const float* wv, const float* bv, const float* w1t, const float* b1,
                  const float* w2, const float* b2, int P, float* pf, float* vout, float* x0ws, float* out,
                  void* stream);

#ifdef __cplusplus
}
#endif
#endif /* BLOKUS_ENGINE_H */
