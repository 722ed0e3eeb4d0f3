/*
 * polarcub_sc.h -- C ABI of the MI355X (gfx950) polar SC hot path.
 *
 * This is the drop-in boundary for the reference's decode path.  The
 * reference (benjilieber/polarcub) is pure Python; the functions below are
 * what its per-codeword calls become when batched:
 *
 *   pcub_sc_decode_bin   replaces BinaryPolarEncoderDecoder.decode
 *                        (BinaryPolarEncoderDecoder.py:71-99) and the recursion it
 *                        drives (:223-325) over BinaryMemorylessVectorDistribution
 *                        (VectorDistributions/BinaryMemorylessVectorDistribution.py:15-87),
 *                        for a uniform a-priori distribution.
 *   pcub_sc_decode_qary  replaces QaryPolarEncoderDecoder.decode
 *                        (QaryPolarEncoderDecoder.py:90-116, :318-401) over
 *                        QaryMemorylessVectorDistribution (:26-118).
 *   pcub_polar_encode_bin replaces BinaryPolarEncoderDecoder.encode
 *                        (BinaryPolarEncoderDecoder.py:46-69) for a uniform prior.
 *   pcub_pack_bits / pcub_unpack_bits / pcub_transpose_pairs: layout helpers.
 *
 * Conventions
 *   - All data pointers are DEVICE pointers (hipMalloc'd or torch CUDA tensors).
 *   - `stream` is a hipStream_t passed as void* (NULL = default stream); every
 *     call is stream-ordered and asynchronous; no call synchronises, and none
 *     allocates except pcub_polar_encode_bin for log2N > 14 (stream-ordered scratch).
 *   - Bit vectors are "word-major, codeword-minor": word w of codeword b is at
 *     words[w * B + b] (32 bits per word, bit t = element 32w+t).  This is the
 *     coalesced layout for one-codeword-per-lane kernels.
 *   - Joint probabilities use the "element-major" layout: xy[(i * B + b) * 2 + x]
 *     = P(X_i = x, Y_i = y_i) of codeword b (binary), i.e. a [N][B][2] array.
 *     pcub_transpose_pairs converts from the reference's per-codeword [B][N][2].
 *   - Return value: 0 on success, PCUB_EINVAL (-1) for invalid arguments,
 *     otherwise the hipError_t of the failed launch.
 *   - Arithmetic contract: IEEE binary64 in the reference's operation order;
 *     decisions are bit-identical to the reference for finite, non-negative
 *     inputs (zeros, subnormals and exact ties included).
 */
#ifndef POLARCUB_SC_H
#define POLARCUB_SC_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define PCUB_EINVAL (-1)

/* Library version, for the loader's ABI check.  3: the deletion state tables carry an 8-double
 * header (size them with pcub_sc_deletion_table_bytes, never from the version-2 formula), and
 * pcub_tile_pairs.  4: pcub_scl_set_wave (the list decoder's slower wave-per-codeword layout) removed. */
int pcub_abi_version(void);

/* Bytes of device workspace pcub_sc_decode_bin needs for a batch of B
 * codewords of length 2^log2N (0 for invalid arguments).  The workspace holds
 * the per-slot SC stage buffers; it is sized by the resident grid, not by B. */
size_t pcub_sc_decode_bin_workspace(int64_t B, int32_t log2N);

/* Binary SC decode of B codewords, uniform a-priori distribution.
 *   xy          [N][B][2] f64 joint probabilities (never modified)
 *   frozen_mask ceil(N/32) u32 words, bit i set <=> u_i frozen
 *   frozen_val  ceil(N/32) u32 words, value of each frozen u_i
 *               (reference: 0 if 0.5 >= r_i else 1, BinaryPolarEncoderDecoder.py:258-262)
 *   K           number of information positions (N - popcount(frozen_mask))
 *   info_words  out, ceil(K/32) x B words: decoded information bits in u order
 *   xhat_words  out, ceil(N/32) x B words: re-encoded codeword estimate (may be NULL)
 *   u_words     out, ceil(N/32) x B words: all N decisions u_0..u_{N-1} (may be NULL)
 *   workspace   device buffer of pcub_sc_decode_bin_workspace(B, log2N) bytes */
int pcub_sc_decode_bin(const double* xy, int64_t B, int32_t log2N, const uint32_t* frozen_mask,
                       const uint32_t* frozen_val, int32_t K, uint32_t* info_words, uint32_t* xhat_words,
                       uint32_t* u_words, void* workspace, size_t workspace_bytes, void* stream);

/* The same decode with the root rows in tiles of T codewords: xy [ceil(B/T)][N][T][2] f64, codeword b's
 * row i at ((b / T) N + i) T + b % T (the last tile's padding columns are never read).  With T =
 * pcub_sc_bin_tile(log2N) -- the codewords one wave of the kernel decodes -- each wave reads its
 * codewords' rows as one contiguous block instead of 2N rows 16 B wide spread B * 16 bytes apart
 * (N = 1024: 78 vs 75 M codewords/s).  T = 0 is the [N][B][2] layout of pcub_sc_decode_bin. */
int pcub_sc_bin_tile(int32_t log2N);
int pcub_sc_decode_bin_tiled(const double* xy, int64_t B, int32_t log2N, int32_t tile, const uint32_t* frozen_mask,
                             const uint32_t* frozen_val, int32_t K, uint32_t* info_words, uint32_t* xhat_words,
                             uint32_t* u_words, void* workspace, size_t workspace_bytes, void* stream);

/* q-ary SC decode (linear domain), 2 <= q <= 8, N >= 4.
 *   xy        [N][B][q] f64 joint probabilities P(X_i = x, Y_i = y_i)
 *   frozen    [N] u8 (1 = frozen; frozen symbols are 0, QaryPolarEncoderDecoder.py:351)
 *   info      out [K][B] u8 decoded information symbols in u order
 *   xhat      out [N][B] u8 re-encoded codeword estimate (may be NULL)
 *   workspace pcub_sc_decode_qary_workspace(B, log2N, q) bytes */
size_t pcub_sc_decode_qary_workspace(int64_t B, int32_t log2N, int32_t q);
int pcub_sc_decode_qary(const double* xy, int64_t B, int32_t log2N, int32_t q, const uint8_t* frozen, int32_t K,
                        uint8_t* info, uint8_t* xhat, void* workspace, size_t workspace_bytes, void* stream);
/* ... with the rows in tiles of T codewords ([ceil(B/T)][N][T][q], as pcub_sc_decode_bin_tiled);
 * pcub_sc_qary_tile: the codewords one wave of the kernel decodes (the native T). */
int pcub_sc_qary_tile(int32_t q, int32_t log2N);
int pcub_sc_decode_qary_tiled(const double* xy, int64_t B, int32_t log2N, int32_t q, int32_t tile,
                              const uint8_t* frozen, int32_t K, uint8_t* info, uint8_t* xhat, void* workspace,
                              size_t workspace_bytes, void* stream);

/* q-ary polar encoder (QaryPolarEncoderDecoder.py:65-88, frozen symbols 0):
 *   info [K][B] u8 -> x [N][B] u8, combine x[2h] = (xm+xp)%q, x[2h+1] = (q-xp)%q. */
int pcub_polar_encode_qary(const uint8_t* info, int64_t B, int32_t log2N, int32_t q, const uint8_t* frozen, int32_t K,
                           uint8_t* x, void* stream);

/* Polar encoder (uniform prior): u_i = frozen_val_i at frozen positions, the
 * next information bit elsewhere; x = polar transform of u in the reference's
 * adjacent-pair convention (BinaryPolarEncoderDecoder.py:319-323, :494-516).
 *   info_words ceil(K/32) x B, x_words out ceil(N/32) x B. */
int pcub_polar_encode_bin(const uint32_t* info_words, int64_t B, int32_t log2N, const uint32_t* frozen_mask,
                          const uint32_t* frozen_val, int32_t K, uint32_t* x_words, void* stream);

/* SC decode over the deletion channel (uniform input): replaces
 * BinaryPolarEncoderDecoder.decode (BinaryPolarEncoderDecoder.py:71-99) over the
 * CollectionOfBinaryTrellises that buildCollectionOfBinaryTrellises_uniformInput_deletion
 * (VectorDistributions/CollectionOfBinaryTrellises.py:106-129, BinaryTrellis.py:309-438,
 * Guardbands.py:47-93) builds from each received word.
 *   rx          [B][stride] u8 received symbols (0/1), rx_len[b] <= stride of them valid
 *   n, n0       code length 2^n, 2^n0 inputs per trellis; supported (decode):
 *               1 <= n0 <= 4, 1 <= n - n0 <= 8 (decode and leaf export), and n0 = 4 with
 *               n - n0 = 9, 10 without ones (decode; main_deletion's n = 13, 14)
 *               (pcub_sc_deletion_supported / pcub_sc_leaf_deletion_supported)
 *   ones        numberOfOnesToAddAtBothEndsOfGuardbands, 0 <= ones <= 3
 *   pd          deletion probability the trellises are built with
 *   frozen_mask / frozen_val / K / info_words / xhat_words as pcub_sc_decode_bin. */
int pcub_sc_deletion_supported(int32_t n, int32_t n0, int32_t ones);
int pcub_sc_leaf_deletion_supported(int32_t n, int32_t n0, int32_t ones);
int pcub_sc_decode_deletion(const uint8_t* rx, const int32_t* rx_len, int64_t B, int32_t stride, int32_t n, int32_t n0,
                            int32_t ones, double pd, const uint32_t* frozen_mask, const uint32_t* frozen_val,
                            int32_t K, uint32_t* info_words, uint32_t* xhat_words, void* stream);

/* Leaf export (LLR check, genie construction).  Decodes like pcub_sc_decode_bin /
 * pcub_sc_decode_deletion (identical decisions) and also writes, for every u index i,
 * the normalised xy leaf node the reference passes to calcMarginalizedProbabilities
 * (BinaryPolarEncoderDecoder.py:250-252, 268-273; the genie's marginalizedUProbs),
 * as a compact value in leaf[i * B + b]: +r = (1, r), -r = (r, 1), NaN = (0, 0).
 * No rate-0 subtree is skipped.  frozen_val_cw ([ceil(N/32)][B] words, may be NULL)
 * gives per-codeword frozen values (the genie's per-trial common randomness,
 * BinaryPolarEncoderDecoder.py:101-112) and then overrides frozen_val.
 * info_words / xhat_words may be NULL.  pcub_sc_leaf_bin needs log2N >= 1 and a
 * workspace of pcub_sc_leaf_bin_workspace(B, log2N) bytes. */
size_t pcub_sc_leaf_bin_workspace(int64_t B, int32_t log2N);
int pcub_sc_leaf_bin(const double* xy, int64_t B, int32_t log2N, const uint32_t* frozen_mask, const uint32_t* frozen_val,
                     const uint32_t* frozen_val_cw, int32_t K, uint32_t* info_words, uint32_t* xhat_words, double* leaf,
                     void* workspace, size_t workspace_bytes, void* stream);
int pcub_sc_leaf_deletion(const uint8_t* rx, const int32_t* rx_len, int64_t B, int32_t stride, int32_t n, int32_t n0,
                          int32_t ones, double pd, const uint32_t* frozen_mask, const uint32_t* frozen_val,
                          const uint32_t* frozen_val_cw, int32_t K, uint32_t* info_words, uint32_t* xhat_words,
                          double* leaf, void* stream);

/* Segment-state tables (n0 = 2: 4 KiB; n0 = 3: 1 MiB; ones = 0): every value a trellis hands to
 * the memoryless subtree is a function of its segment (m <= 2^n0 received bits) and of the bits
 * the subtree returned before it, so one table per pd replaces the per-lane trellis levels
 * (DESIGN 3.2).  pcub_sc_deletion_table_bytes(n0) is its size (0: no table for n0);
 * pcub_sc_deletion_build_table fills it on the stream (8-byte aligned device memory).
 * The _tab twins of the two deletion entry points read it when n0 = 2 or 3 and ones = 0 and the
 * table was built for the same n0 and pd (its header); otherwise, or with table = NULL, they decode
 * as the plain entry points (n0 = 2 then builds its table per workgroup).  Decisions are
 * identical either way.  The table must stay allocated and unmodified while decodes that read it
 * are in flight (ordinary stream rules: build and decode on one stream, or synchronise).  Every
 * kernel checks the table's header (magic, n0, pd) on the device before reading it; a rejected
 * table sends the batch to the table-less path. */
int64_t pcub_sc_deletion_table_bytes(int32_t n0);
/* Diagnostics: allow (1, the default) or forbid (0) the table-driven layout, 16 lanes per codeword
 * (DESIGN 3.2); returns the previous setting.  Decisions are identical either way. */
int pcub_sc_set_deletion_dense(int32_t on);
/* Tuning hook: lanes a codeword of that layout, 8 (default) or 16, or 4 (up to 64 trellises; 8
 * beyond); returns the previous value, -1 for another value.  Decisions are identical either way. */
int pcub_sc_set_deletion_lanes(int32_t lanes);
/* 1 when pcub_sc_decode_deletion_tab would run the table-driven layout for this shape, received
 * row stride, table and pd (diagnostics: which kernel a profile names). */
int pcub_sc_deletion_dense_layout(int32_t n, int32_t n0, int32_t ones, int32_t stride, const double* table, double pd);
int pcub_sc_deletion_build_table(int32_t n0, double pd, double* table, void* stream);
int pcub_sc_decode_deletion_tab(const uint8_t* rx, const int32_t* rx_len, int64_t B, int32_t stride, int32_t n,
                                int32_t n0, int32_t ones, double pd, const uint32_t* frozen_mask,
                                const uint32_t* frozen_val, int32_t K, uint32_t* info_words, uint32_t* xhat_words,
                                const double* table, void* stream);
int pcub_sc_leaf_deletion_tab(const uint8_t* rx, const int32_t* rx_len, int64_t B, int32_t stride, int32_t n,
                              int32_t n0, int32_t ones, double pd, const uint32_t* frozen_mask,
                              const uint32_t* frozen_val, const uint32_t* frozen_val_cw, int32_t K,
                              uint32_t* info_words, uint32_t* xhat_words, double* leaf, const double* table,
                              void* stream);
/* q-ary SC in the log domain (QaryPolarEncoderDecoder(..., use_log=True).decode,
 * QaryPolarEncoderDecoder.py:318-401 over VectorDistributions/QaryMemorylessVectorDistribution.py
 * with use_log): logaddexp minus transform, logsumexp normalisation and marginal.
 *   xy    [N][B][q] f64 log-probabilities (-inf allowed); q in 2..8, log2N in 1..16
 *   info  [K][B] u8 symbols; xhat [N][B] u8 or NULL; leaf [N][B][q] f64 log marginals or NULL
 * Device exp/log1p/log: values agree with the reference within a few ulps (not bit-exact).
 * Workspace: pcub_sc_decode_qary_log_workspace(B, q, log2N) bytes. */
size_t pcub_sc_decode_qary_log_workspace(int64_t B, int32_t q, int32_t log2N);
int pcub_sc_decode_qary_log(const double* xy, int64_t B, int32_t q, int32_t log2N, const uint32_t* frozen_mask,
                            int32_t K, uint8_t* info, uint8_t* xhat, double* leaf, void* workspace,
                            size_t workspace_bytes, void* stream);

/* q-ary SCL / Fast-SSC list decoding (QaryPolarEncoderDecoder.listDecode,
 * QaryPolarEncoderDecoder.py:118-227, 403-820; rate-0, repetition, rate-1 and single-parity-check
 * nodes as the reference), linear domain, one lane per codeword.
 *   xy           [N][B][q] f64; q in 2..8, log2N in 0..12, L (maxListSize) in 1..64
 *   frozen       [N] u8 (1 = frozen); frozen_vals [nF][B] u8 frozen values in frozen-index order
 *   actual       [K][B] u8 actual information (listDecode's actualInformation) or NULL
 *   out_info     [L][K][B] u8 final list (rows >= out_size: 0xff); out_prob [L][B] f64 metrics
 *                (normalised to max 1); out_size [B]; out_actual [B] actual_prob (with actual)
 * Ties among candidate metrics / reliabilities go to the lower index and the list is kept in
 * ascending candidate order (the reference's order comes from numpy's argpartition, which is
 * CPU-dependent); without ties the final path set and metrics are the reference's.
 * Workspace: pcub_scl_qary_workspace(B, q, log2N, L, K) bytes. */
size_t pcub_scl_qary_workspace(int64_t B, int32_t q, int32_t log2N, int32_t L, int32_t K);
int pcub_scl_qary(const double* xy, int64_t B, int32_t q, int32_t log2N, int32_t L, const uint8_t* frozen,
                  const uint8_t* frozen_vals, int32_t nF, const uint8_t* actual, int32_t K, uint8_t* out_info,
                  double* out_prob, int32_t* out_size, double* out_actual, void* workspace, size_t workspace_bytes,
                  void* stream);

/* The same list decoder in the log domain: QaryPolarEncoderDecoder(..., use_log=True).listDecode,
 * recursiveListDecode's use_log branches (QaryPolarEncoderDecoder.py:403-757, normalize :867-872).
 * xy holds log-probabilities; out_prob / out_actual are log-domain metrics (the largest is 0).
 * Transforms by numpy's logaddexp and scipy's logsumexp as pcub_sc_decode_qary_log, metrics add,
 * the products of the linear domain become the reference's sums (np.sum's pairwise order over a
 * node's positions).  exp / log1p / log are the device's: values agree with the reference to a few
 * ulps.  Same arguments, workspace and tie rules as pcub_scl_qary. */
int pcub_scl_qary_log(const double* xy, int64_t B, int32_t q, int32_t log2N, int32_t L, const uint8_t* frozen,
                      const uint8_t* frozen_vals, int32_t nF, const uint8_t* actual, int32_t K, uint8_t* out_info,
                      double* out_prob, int32_t* out_size, double* out_actual, void* workspace,
                      size_t workspace_bytes, void* stream);

/* Non-uniform a-priori distribution (two trees).  Replaces recursiveEncodeDecode with an
 * xVectorDistribution that is not uniform (BinaryPolarEncoderDecoder.py:223-325, called by
 * decode :71-99 and encode :46-69): the prior tree px runs beside the xy tree through the same
 * minus / plus / max-normalise steps; a frozen u_i = 0 iff the prior leaf's marginal
 * m0 >= rnd[i] (:258-262), an information u_i is the xy leaf's decision (:249-252).
 *   xy          [N][B][2] f64 joint pairs (decode), or NULL to encode: the information bits
 *               are then READ from info_words and only the prior tree runs (:254)
 *   px          [N][px_batch][2] f64 prior pairs, px_batch = 1 (one prior for the batch) or B
 *   rnd         [N] f64 common randomness (randomlyGeneratedNumbers, :33-44)
 *   leaf        NULL or [N][B] compact leaves of the deciding tree (xy; prior when encoding)
 *               -- marginalizedUProbs (:267-273)
 *   info_words  [ceil(K/32)][B]: written (decode) or read (encode); xhat_words may be NULL.
 * log2N in 1..20; workspace of pcub_sc_prior_bin_workspace(B, log2N) bytes. */
size_t pcub_sc_prior_bin_workspace(int64_t B, int32_t log2N);
int pcub_sc_prior_bin(const double* xy, const double* px, int64_t px_batch, int64_t B, int32_t log2N,
                      const uint32_t* frozen_mask, const double* rnd, int32_t K, uint32_t* info_words,
                      uint32_t* xhat_words, double* leaf, void* workspace, size_t workspace_bytes, void* stream);

/* compact leaves -> the reference's marginals (calcMarginalizedProbabilities,
 * VectorDistributions/BinaryMemorylessVectorDistribution.py:52-69): s = p0 + p1,
 * m = p / s, (0.5, 0.5) when s = 0.  count values in, [count][2] f64 out. */
int pcub_leaf_marginals(const double* leaf, int64_t count, double* marginals, void* stream);

/* Binary SC decode of compact normalised rows: xc [N][B] f64, +r standing for the joint row
 * (1, r) and -r for (r, 1) (NaN: (0, 0)).  The same decode as pcub_sc_decode_bin on those pairs
 * (the reference's arithmetic on a row with a 1 in it is the compact one), from 8 bytes a position
 * instead of 16.  Workspace: pcub_sc_decode_bin_compact_workspace(B, log2N) bytes.
 * pcub_sc_decode_bin_compact_direct(log2N): 1 when that code length runs a compact-root kernel,
 * 0 when the call expands the rows into pairs in its workspace first (B * N * 16 more bytes). */
int pcub_sc_decode_bin_compact_direct(int32_t log2N);
size_t pcub_sc_decode_bin_compact_workspace(int64_t B, int32_t log2N);
int pcub_sc_decode_bin_compact(const double* xc, int64_t B, int32_t log2N, const uint32_t* frozen_mask,
                               const uint32_t* frozen_val, int32_t K, uint32_t* info_words, uint32_t* xhat_words,
                               uint32_t* u_words, void* workspace, size_t workspace_bytes, void* stream);
/* ... with the rows in tiles of T codewords ([ceil(B/T)][N][T] f64; workspace for the padded batch:
 * pcub_sc_decode_bin_compact_workspace(ceil(B/T) T, log2N)). */
int pcub_sc_decode_bin_compact_tiled(const double* xc, int64_t B, int32_t log2N, int32_t tile,
                                     const uint32_t* frozen_mask, const uint32_t* frozen_val, int32_t K,
                                     uint32_t* info_words, uint32_t* xhat_words, uint32_t* u_words, void* workspace,
                                     size_t workspace_bytes, void* stream);

/* Device Monte-Carlo (encodeDecodeSimulation, BinaryPolarEncoderDecoder.py:328-387, as a
 * batched pipeline).  Codeword g's draws come from Philox4x32-10 keyed by (seed, g), so
 * the codewords [offset, offset + B) are identical whichever rank or chunk makes them.
 *   pcub_mc_info     K uniform information bits per codeword -> [ceil(K/32)][B] words
 *   pcub_mc_channel  codeword bits [ceil(N/32)][B] -> joint pairs [N][B][2] f64;
 *                    channel 0 = BI-AWGN (param = sigma^2, BPSK 0 -> +1),
 *                    channel 1 = BSC (param = p, makeBSC's table)
 *   pcub_mc_channel_norm  normalised rows (each divided by its larger entry: the same channel law;
 *                    four elements a Philox counter, the row arithmetic in f32), compact
 *                    ([N][B] f64, compact != 0) or as pairs
 *   pcub_mc_count_errors  counters[0] += B, [1] += frame errors, [2] += bit errors
 *   pcub_mc_run_bin  info -> encode -> channel (normalised, compact) -> decode -> count for codewords
 *                    [offset, offset + count), chunk codewords at a time; counters
 *                    (device u64[4]) accumulate; the caller zeroes them. */
int pcub_mc_info(uint64_t seed, int64_t offset, int64_t B, int32_t K, uint32_t* info_words, void* stream);
int pcub_mc_channel(uint64_t seed, int64_t offset, int64_t B, int32_t log2N, int32_t channel, double param,
                    const uint32_t* x_words, double* xy, void* stream);
int pcub_mc_channel_norm(uint64_t seed, int64_t offset, int64_t B, int32_t log2N, int32_t channel, double param,
                         const uint32_t* x_words, double* out, int32_t compact, void* stream);
/* the same rows written in tiles of T codewords (pcub_sc_decode_bin_tiled's layout; T = 0: [N][B]) */
int pcub_mc_channel_tiled(uint64_t seed, int64_t offset, int64_t B, int32_t log2N, int32_t channel, double param,
                          const uint32_t* x_words, double* xy, int32_t tile, void* stream);
int pcub_mc_channel_norm_tiled(uint64_t seed, int64_t offset, int64_t B, int32_t log2N, int32_t channel, double param,
                               const uint32_t* x_words, double* out, int32_t compact, int32_t tile, void* stream);
int pcub_mc_count_errors(const uint32_t* decoded_words, const uint32_t* sent_words, int64_t B, int32_t K,
                         uint64_t* counters, void* stream);
size_t pcub_mc_run_bin_workspace(int64_t chunk, int32_t log2N, int32_t K);

/* The q-ary and deletion Monte-Carlo inputs under the same global-index keying (so q-ary and
 * deletion runs sharded over G GPUs decode the 1-GPU run's codewords and their counters match):
 *   pcub_mc_info_qary    K uniform symbols in [0, q) per codeword -> [K][B] u8
 *   pcub_mc_channel_qsc  q-ary codewords [N][B] u8 -> QSC(p) joint rows [N][B][q] f64
 *                        (makeQSC, ScalarDistributions/QaryMemorylessDistribution.py:780-784)
 *   pcub_mc_deletion     codeword bits [ceil(N/32)][B] -> the guard-banded word of template tmpl
 *                        (W entries: >= 0 a codeword bit index, -1 a guard zero, -2 a guard one;
 *                        Guardbands.addDeletionGuardBands, Guardbands.py:4-44) through the
 *                        deletion channel (each symbol dropped with probability pd,
 *                        BinaryTrellis.deletionChannelSimulation, BinaryTrellis.py:441-461):
 *                        rx [B][W] u8 (survivors left-packed, zero-padded), rx_len [B] i32 */
int pcub_mc_info_qary(uint64_t seed, int64_t offset, int64_t B, int32_t K, int32_t q, uint8_t* info, void* stream);
int pcub_mc_channel_qsc(uint64_t seed, int64_t offset, int64_t B, int32_t log2N, int32_t q, double p,
                        const uint8_t* x, double* xy, void* stream);
int pcub_mc_channel_qsc_tiled(uint64_t seed, int64_t offset, int64_t B, int32_t log2N, int32_t q, double p,
                              const uint8_t* x, double* xy, int32_t tile, void* stream);
int pcub_mc_deletion(uint64_t seed, int64_t offset, int64_t B, int32_t log2N, const int32_t* tmpl, int32_t W,
                     double pd, const uint32_t* x_words, uint8_t* rx, int32_t* rx_len, void* stream);

int pcub_mc_run_bin(uint64_t seed, int64_t offset, int64_t count, int32_t log2N, int32_t channel, double param,
                    const uint32_t* frozen_mask, const uint32_t* frozen_val, int32_t K, int64_t chunk,
                    uint64_t* counters, void* workspace, size_t workspace_bytes, void* stream);

/* mc_run for the q-ary and deletion workloads: the chained generators above, the decode and the
 * counters for codewords [offset, offset + count), chunk at a time, on the stream.  counters
 * (device u64[4], the caller zeroes them) accumulate [0] codewords, [1] frame errors, [2] symbol
 * (q-ary) or information-bit (deletion) errors.
 *   pcub_mc_run_qary      info (pcub_mc_info_qary) -> pcub_polar_encode_qary -> QSC(p) rows in the
 *                         decode's tiles -> pcub_sc_decode_qary_tiled -> symbol errors
 *                         (QaryPolarEncoderDecoder.py:935-982's trial loop)
 *   pcub_mc_run_deletion  info -> pcub_polar_encode_bin -> pcub_mc_deletion (template tmpl of W
 *                         entries, channel pd) -> pcub_sc_decode_deletion_tab (stride W, trellises
 *                         built with the same pd; table as there, may be NULL) -> bit errors
 *                         (main_deletion.py:142-146's trial loop)
 * Workspaces: pcub_mc_run_qary_workspace(chunk, log2N, q, K), pcub_mc_run_deletion_workspace(chunk,
 * n, W, K) bytes. */
size_t pcub_mc_run_qary_workspace(int64_t chunk, int32_t log2N, int32_t q, int32_t K);
int pcub_mc_run_qary(uint64_t seed, int64_t offset, int64_t count, int32_t log2N, int32_t q, double p,
                     const uint8_t* frozen, int32_t K, int64_t chunk, uint64_t* counters, void* workspace,
                     size_t workspace_bytes, void* stream);
size_t pcub_mc_run_deletion_workspace(int64_t chunk, int32_t n, int32_t W, int32_t K);
int pcub_mc_run_deletion(uint64_t seed, int64_t offset, int64_t count, int32_t n, int32_t n0, const int32_t* tmpl,
                         int32_t W, int32_t ones, double pd, const uint32_t* frozen_mask, const uint32_t* frozen_val,
                         int32_t K, const double* table, int64_t chunk, uint64_t* counters, void* workspace,
                         size_t workspace_bytes, void* stream);

/* [B][nbits] u8 (0/1) -> ceil(nbits/32) x B words, and back. */
int pcub_pack_bits(const uint8_t* bits, int64_t B, int32_t nbits, uint32_t* words, void* stream);
int pcub_unpack_bits(const uint32_t* words, int64_t B, int32_t nbits, uint8_t* bits, void* stream);

/* [B][N][q] f64 -> [N][B][q] f64, 1 <= q <= 8 (q = 2 for binary pairs). */
int pcub_transpose_pairs(const double* src, int64_t B, int32_t N, int32_t q, double* dst, void* stream);

/* [B][N][q] f64 -> the tiled layout [ceil(B/T)][N][T][q] f64 that pcub_sc_decode_bin_tiled /
 * pcub_sc_decode_qary_tiled read (codeword b's row i at ((b / T) N + i) T + b % T; the last tile's
 * padding columns zero), 1 <= q <= 8, 1 <= T <= 4096: the reference's per-codeword rows
 * (BinaryMemorylessVectorDistribution.probs) in one pass into the layout the headline kernel reads. */
int pcub_tile_pairs(const double* src, int64_t B, int32_t N, int32_t q, int32_t T, double* dst, void* stream);

#ifdef __cplusplus
}
#endif

#endif /* POLARCUB_SC_H */
