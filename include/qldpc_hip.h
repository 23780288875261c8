/*
 * qldpc_hip.h — C ABI of the MI355X (gfx950) Monte Carlo BP decoding engine.
 *
 * The reference's hot path is Python calling the third-party `ldpc`
 * bp_decoder once per shot.  Each entry point below replaces
 * one reference interface; the Python host layer (qldpc_fault_tolerance_amd/)
 * binds them with ctypes exactly as INTEGRATION.md shows.
 *
 * Conventions: every function returns 0 on success or a negative error code
 * (see QLDPC_E*), and qldpc_last_error() returns a thread-local message.
 * Device pointers (d_*) are plain device addresses (e.g. torch
 * Tensor.data_ptr()); `stream` is a hipStream_t passed as void* (NULL = the
 * legacy default stream).  Handles are not thread-safe: one host thread per
 * handle; distinct handles may be used concurrently.
 */
#ifndef QLDPC_HIP_H
#define QLDPC_HIP_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define QLDPC_ABI_VERSION 1

#define QLDPC_OK 0
#define QLDPC_EINVAL -1   /* bad argument (shape, range, NULL)            */
#define QLDPC_EHIP -2     /* HIP runtime error (message has hipGetErrorString) */
#define QLDPC_ENOMEM -3   /* allocation failed                            */
#define QLDPC_ENOTSUP -4  /* graph/method combination not supported       */

/* bp_method, as the strings the reference passes (src/Decoders.py:80-84) */
#define QLDPC_PRODUCT_SUM 0
#define QLDPC_MIN_SUM 1

/* logical_mode = eval_logical_type of CodeSimulator_DataError (src/Simulators.py:162-168) */
#define QLDPC_LOGICAL_X 0
#define QLDPC_LOGICAL_Z 1
#define QLDPC_LOGICAL_TOTAL 2

#define QLDPC_HIST_BINS 1025 /* iteration histogram bins (iter 0..1024; last bin = >=1024) */

typedef struct qldpc_graph qldpc_graph;
typedef struct qldpc_bp qldpc_bp;
typedef struct qldpc_mc qldpc_mc;
typedef struct qldpc_phenl qldpc_phenl;

/* Counters of one fused Monte Carlo run (summed over calls if not reset). */
typedef struct {
  int64_t shots;               /* shots simulated                                */
  int64_t failures;            /* shots whose eval_logical_type outcome failed   */
  int64_t sector_decodes[2];   /* [0] = X errors on hz, [1] = Z errors on hx      */
  int64_t sector_iters[2];     /* sum of BP iterations                            */
  int64_t sector_nonconv[2];   /* decodes that hit max_iter without H x == s      */
  int64_t sector_fail[2];      /* sector failures (syndrome mismatch or logical)  */
  int64_t iter_hist[2][QLDPC_HIST_BINS];
} qldpc_counters;

int qldpc_abi_version(void);
const char *qldpc_last_error(void);
int qldpc_device_count(int *out);

/* Build flags of this library: QLDPC_BUILD_EXPERIMENTAL when the measured-and-not-kept kernel
 * families (c2s 31103, m2v 40103, fp64 257-512 threads 303, engine 4) are compiled in
 * (-DQLDPC_EXPERIMENTAL=1); the product build leaves them out and ignores their opt-ins. */
#define QLDPC_BUILD_EXPERIMENTAL 1
int qldpc_build_flags(void);

/*
 * Tanner graph of a parity-check matrix H (m x n), CSR with columns ascending
 * inside each row (the `mod2sparse` order `ldpc` builds from the ndarray it is
 * given: src/Decoders.py:80, `bp_decoder(parity_check_matrix=h, ...)`).
 * Copied to the device; the caller's arrays may be freed after the call.
 */
int qldpc_graph_create(int device, int32_t m, int32_t n, const int32_t *row_ptr, const int32_t *col_idx,
                       qldpc_graph **out);
int qldpc_graph_destroy(qldpc_graph *g);
int qldpc_graph_info(const qldpc_graph *g, int32_t *m, int32_t *n, int32_t *nnz, int32_t *max_row_deg,
                     int32_t *max_col_deg);

/*
 * BP decoder on a graph: replaces `ldpc.bp_decoder(parity_check_matrix=h,
 * channel_probs=..., max_iter=..., bp_method=..., ms_scaling_factor=...)`
 * (src/Decoders.py:80-84, :52-56; src/Decoders_SpaceTime.py:207-213).
 *   channel_probs : host array of n doubles (priors log((1-p)/p) computed on
 *                   the host with libm, as the Cython does);
 *   max_iter      : <= 0 means n (ldpc's default);
 *   ms_scaling_factor : alpha; 0 selects alpha = 1 - 2^-iter;
 *   precision     : 64 = float64 messages (reference arithmetic, bit-exact
 *                   with the oracle), 32 = float32 fast mode (same op order).
 *   vars_per_thread : 0 = automatic; else variables per thread (tuning knob).
 *   min_col_slots : 0 = automatic; else edge slots per variable are at least
 *                   this (4 or 8) — lets the two sectors of one MC run share a
 *                   kernel variant when hx and hz have different column degrees.
 */
int qldpc_bp_create(qldpc_graph *g, const double *channel_probs, int32_t max_iter, int32_t bp_method,
                    double ms_scaling_factor, int32_t precision, int32_t vars_per_thread, int32_t min_col_slots,
                    qldpc_bp **out);
int qldpc_bp_destroy(qldpc_bp *bp);
int qldpc_bp_set_channel_probs(qldpc_bp *bp, const double *channel_probs);

/*
 * Decode B syndromes: the batched form of `bp_decoder.decode(synd)` (and
 * BPDecoder.decode, src/Decoders.py:88-90).
 *   d_synd  : uint8 [B][m] 0/1          d_corr : uint8 [B][n] 0/1 (output)
 *   d_iters : int32 [B] or NULL         d_conv : uint8 [B] or NULL
 */
int qldpc_bp_decode_batch(qldpc_bp *bp, const uint8_t *d_synd, uint8_t *d_corr, int32_t *d_iters,
                          uint8_t *d_conv, int64_t B, void *stream);

/*
 * Soft-output BP for BP+OSD (src/Decoders.py:26-41: `bposd_decoder` runs
 * ldpc's BP, then OSD on its final `log_prob_ratios` when BP did not converge).
 * qldpc_bp_create_soft builds a min-sum decoder on engine 1 (the kernel that
 * can write posteriors); qldpc_bp_decode_batch_soft is qldpc_bp_decode_batch
 * plus d_post: double [B][n] = the last iteration's posterior log-probability
 * ratios (ldpc's log_prob_ratios; exact fp32 values widened in fp32 mode).
 * A product-sum decoder (qldpc_bp_create with bp_method 0, engine 5) takes
 * qldpc_bp_decode_batch_soft too: d_post = ldpc bp_decode_prob_ratios'
 * log_prob_ratios = log(1 / posterior ratio) in double (the device's log: equal
 * to libm's except for rare 1-ulp differences).
 */
int qldpc_bp_create_soft(qldpc_graph *g, const double *channel_probs, int32_t max_iter, double ms_scaling_factor,
                         int32_t precision, qldpc_bp **out);
int qldpc_bp_decode_batch_soft(qldpc_bp *bp, const uint8_t *d_synd, uint8_t *d_corr, int32_t *d_iters,
                               uint8_t *d_conv, double *d_post, int64_t B, void *stream);

/*
 * Ordered-statistics decoding (the OSD half of `bposd_decoder(h,
 * channel_probs, max_iter, bp_method, ms_scaling_factor, osd_method,
 * osd_order)`, src/Decoders.py:29-36; BPOSD_Decoder.decode returns
 * `osdw_decoding`, :39-41).  Host-side stage (GF(2) elimination per
 * non-converged syndrome, std::thread pool); all pointers are HOST pointers.
 *   osd_method : 0 = "osd_0", 1 = "osd_e" (exhaustive over 2^osd_order
 *                inputs; the reference's choice), 2 = "osd_cs";
 *   decode     : synd uint8 [B][m], post double [B][n] (BP posteriors), conv
 *                uint8 [B] or NULL (converged shots copy bp_corr [B][n]),
 *                out_osd0 (or NULL) / out_osdw uint8 [B][n];
 *   threads    : <= 0 = OMP_NUM_THREADS if set, else all hardware threads.
 */
typedef struct qldpc_osd qldpc_osd;
int qldpc_osd_create(int32_t m, int32_t n, const int32_t *row_ptr, const int32_t *col_idx,
                     const double *channel_probs, int32_t osd_method, int32_t osd_order, qldpc_osd **out);
int qldpc_osd_destroy(qldpc_osd *osd);
int qldpc_osd_rank(const qldpc_osd *osd, int32_t *rank);
int qldpc_osd_decode_batch(const qldpc_osd *osd, const uint8_t *synd, const double *post, const uint8_t *conv,
                           const uint8_t *bp_corr, uint8_t *out_osd0, uint8_t *out_osdw, int64_t B,
                           int32_t threads);

/*
 * GPU OSD (n <= 8192, osd_e order <= 24): the same outputs as qldpc_osd_decode_batch, one
 * workgroup per syndrome; all pointers are DEVICE pointers (d_post from
 * qldpc_bp_decode_batch_soft).  Uniform channel_probs weigh candidates by popcount; non-uniform
 * ones (the circuit-level DEM priors) by sum log(1/p_j), added in ascending column order as the
 * host stage does.
 */
typedef struct qldpc_osd_gpu qldpc_osd_gpu;
int qldpc_osd_gpu_create(const qldpc_graph *g, const double *channel_probs, int32_t osd_method, int32_t osd_order,
                         qldpc_osd_gpu **out);
int qldpc_osd_gpu_destroy(qldpc_osd_gpu *osd);
int qldpc_osd_gpu_decode(qldpc_osd_gpu *osd, const uint8_t *d_synd, const double *d_post, const uint8_t *d_conv,
                         const uint8_t *d_bp_corr, uint8_t *d_out0, uint8_t *d_outw, int64_t B, void *stream);
/*
 * FirstMinBPDecoder (src/Decoders.py:49-74) on the device: one-iteration min-sum BP (ldpc
 * bp_decoder, max_iter = 1, bp_method "minimum_sum") repeated on the running syndrome while the
 * residual syndrome weight does not grow, at most max_iter accepted steps; the corrections are the
 * xor of the accepted steps' decisions.  One workgroup per syndrome, the whole loop on the device.
 *   create : graph g, channel_probs [n] in (0, 1), max_iter, ms_scaling_factor (0 = ldpc's
 *            1 - 2^-iter schedule at iter 1), precision 64 (ldpc's double) or 32; 2 (m + n) <= 64 KiB.
 *   decode : device pointers d_synd [B][m] u8 -> d_corr [B][n] u8, d_steps [B] i32 (accepted
 *            steps, or NULL), on `stream`.
 * Replaces the Python loop of FirstMinBPDecoder.decode (Decoders.py:60-74).
 */
typedef struct qldpc_firstmin qldpc_firstmin;
/* qldpc_phenl_set_round_firstmin (declared after qldpc_phenl below) makes the noisy rounds of the
 * phenomenological pipeline decode with these (CodeSimulator_Phenon with FirstMinBPDecoder decoder1,
 * the Single-Shot notebook's configuration). */
int qldpc_firstmin_create(const qldpc_graph *g, const double *channel_probs, int32_t max_iter,
                          double ms_scaling_factor, int32_t precision, qldpc_firstmin **out);
int qldpc_firstmin_destroy(qldpc_firstmin *fm);
int qldpc_firstmin_decode(qldpc_firstmin *fm, const uint8_t *d_synd, uint8_t *d_corr, int32_t *d_steps, int64_t B,
                          void *stream);

/* Elimination geometry the handle chose (no reference counterpart; tests and DESIGN.md §4):
 * row_words = 64-bit words per register row (0: LDS / HBM image), window_words = the column
 * window's row words (0: none; its overruns are redone at full width), threads = per workgroup,
 * workgroups = the launch's persistent grid (the window launch's when there is one). */
int qldpc_osd_gpu_geometry(const qldpc_osd_gpu *osd, int32_t *row_words, int32_t *window_words, int32_t *threads,
                           int32_t *workgroups);

/*
 * Fused Monte Carlo shot loop = CodeSimulator_DataError._single_run
 * (src/Simulators.py:117-168) for many shots in one launch: per shot sample
 * the Pauli error (3-way split of u, :99-113), syndrome H e, BP decode,
 * residual, failure = (H r != 0) or (L r != 0).
 *   dec_x, logical_x : decoder on hz and the lz logicals (sector X);
 *   dec_z, logical_z : decoder on hx and the lx logicals (sector Z); either
 *                      sector may be NULL if logical_mode does not need it.
 * Shots are keyed by their global index: shot s, qubit j draws
 * u = Philox4x32-10(key = seed, ctr = (j, s_lo, s_hi, stream)) as a 53-bit
 * double, so any shot range sharded over devices reproduces the same counts.
 */
int qldpc_mc_create(qldpc_bp *dec_x, const qldpc_graph *logical_x, qldpc_bp *dec_z,
                    const qldpc_graph *logical_z, qldpc_mc **out);
int qldpc_mc_destroy(qldpc_mc *mc);

/* Async launch: counters accumulate in device memory (d_counters, a
 * qldpc_counters-sized device buffer, zeroed by the caller).  uniforms: NULL
 * => Philox, else device doubles [shot_count][n] (bit-exact replays of an
 * external u stream, e.g. CPython random()).  Optional per-shot outputs
 * (device, NULL to skip): d_fail uint8 [S] (bit0 X-sector fail, bit1 Z),
 * d_err uint8 [S][n] (bit0 x, bit1 z), d_corr uint8 [S][2][n], d_iters
 * int32 [S][2].  grid_blocks <= 0 selects a persistent grid sized to the device.
 */
int qldpc_mc_launch(qldpc_mc *mc, double px, double py, double pz, uint64_t seed, uint64_t shot_begin,
                    int64_t shot_count, int32_t logical_mode, const double *d_uniforms, void *d_counters,
                    uint8_t *d_fail, uint8_t *d_err, uint8_t *d_corr, int32_t *d_iters, int32_t grid_blocks,
                    void *stream);

/* Synchronous convenience: launch + copy counters to host (accumulating into *out). */
int qldpc_mc_run(qldpc_mc *mc, double px, double py, double pz, uint64_t seed, uint64_t shot_begin,
                 int64_t shot_count, int32_t logical_mode, qldpc_counters *out, void *stream);

/*
 * Phenomenological space-time shot loop = CodeSimulator_Phenon_SpaceTime
 * (src/Simulators_SpaceTime.py:382-548): per sample, num_rounds - 1 noisy
 * rounds of num_rep repetitions (fresh depolarizing data error + syndrome
 * flips with probability q, :395-431), each decoded by BP on the stacked
 * space-time graph (ST_BP_Decoder_syndrome, src/Decoders_SpaceTime.py:200-223)
 * from its detector history (Z sector differenced, X sector raw: quirk Q3,
 * :464-476), then a perfect final round decoded by dec2 and the failure check
 * of :500-529.
 *   st_x / st_z   : decoders on GetSpaceTimeCheckMat(hz / hx, num_rep)
 *                   (checked against the final decoders' graphs);
 *   dec2_x/dec2_z : final-round decoders on hz / hx;
 *   logical_x/_z  : lz / lx.
 *   max_batch     : samples in flight per pass (0 = 65536); device buffers
 *                   are sized for it at create time.
 * Both sectors are required (the uniform stream interleaves both check sets).
 */
int qldpc_phenl_create(qldpc_bp *st_x, qldpc_bp *st_z, qldpc_bp *dec2_x, qldpc_bp *dec2_z,
                       const qldpc_graph *logical_x, const qldpc_graph *logical_z, int32_t num_rep, int64_t max_batch,
                       qldpc_phenl **out);
int qldpc_phenl_destroy(qldpc_phenl *ph);
/* Bytes per sample of the optional trace: per noisy round the Z then X
 * detector histories ([num_rep][m_x], [num_rep][m_z]), then the final Z and X
 * syndromes. */
int qldpc_phenl_trace_len(const qldpc_phenl *ph, int32_t num_rounds, int64_t *out);
/* Async launch on `stream`; counters accumulate into d_counters (device
 * qldpc_counters, zeroed by the caller; sector_* count the ST and final
 * decodes).  Sample s uses global index shot_begin + s for its Philox stream,
 * or d_uniforms[s][n_u] (n_u = ((num_rounds-1)*num_rep + 1)*(n + m_x + m_z),
 * CPython's draw order) when non-NULL.  d_fail uint8 [S] (bit0 X, bit1 Z) and
 * d_trace uint8 [S][trace_len] are optional. */
int qldpc_phenl_launch(qldpc_phenl *ph, double px, double py, double pz, double q, uint64_t seed,
                       uint64_t shot_begin, int64_t shot_count, int32_t num_rounds, int32_t logical_mode,
                       const double *d_uniforms, void *d_counters, uint8_t *d_fail, uint8_t *d_trace, void *stream);

/* BP+OSD as the final-round decoder (decoder2 = BPOSD_Decoder in the
 * notebooks, src/Decoders.py:100-138): the sectors given a GPU OSD handle
 * decode the perfect round with soft BP (dec2 must come from
 * qldpc_bp_create_soft) and then OSD where BP did not converge.  NULL = plain
 * BP for that sector.  Declared after qldpc_osd_gpu above. */
int qldpc_phenl_set_final_osd(qldpc_phenl *ph, qldpc_osd_gpu *osd_x, qldpc_osd_gpu *osd_z);
/* Noisy rounds decoded by FirstMinBPDecoder (qldpc_firstmin_*, built on exactly the ST graph of st_x /
 * st_z) instead of BP; NULL keeps BP for that sector.  The trace counters then hold the accepted
 * first-min steps as iterations and count no non-converged decodes for those rounds. */
int qldpc_phenl_set_round_firstmin(qldpc_phenl *ph, qldpc_firstmin *fm_x, qldpc_firstmin *fm_z);

/* Launch geometry chosen for a decoder (threads per shot, vars per thread,
 * LDS bytes, resident blocks per CU) — reported by bench.py / DESIGN.md. */
int qldpc_bp_geometry(const qldpc_bp *bp, int32_t *threads, int32_t *vars_per_thread, int32_t *lds_bytes,
                      int32_t *blocks_per_cu);

/* Kernel engine serving a decoder: 3 = register-resident variables (default
 * when the graph fits: column degree <= 4, <= 8 variables per thread, image
 * < 64 KiB), 2 = streamed variables, 1 = LDS-atomic check state, 4 = engine 3
 * with c2v computed by the check phase, 5 = product-sum (bp_method 0), 6 = HBM-resident
 * messages (qldpc_bp_create_hbm; automatic for images over 160 KiB).
 * QLDPC_ENGINE in the environment selects 1, 2 or 4 explicitly. */
int qldpc_bp_engine(const qldpc_bp *bp, int32_t *engine);

/* Compile-time family of the decoder's kernels (the ENG template argument of rmc_kernel /
 * rdec_kernel as rocprofv3 prints it): engine 3 = 3, 13 (dword-scaled addresses), 103 (fp64
 * <= 256 threads), 303 (fp64 257-512 threads), 1013 (tail layout, 1024 threads), 11103 (fp64
 * m2-in-slot, rows of 3 chunks + a tail slot, 3 workgroups per CU); other engines their number.
 * row_chunks = 16-byte chunks per check row (engines 2-4). */
int qldpc_bp_kernel_id(const qldpc_bp *bp, int32_t *kernel_id, int32_t *row_chunks);

/* Engine 3: leading variable slots per thread that hold only variables of
 * column degree <= 3 (variables are host-sorted by degree; those slots skip the
 * 4th edge slot at compile time).  0 for the other engines and for the fp64
 * kernels of workgroups wider than 256 threads. */
int qldpc_bp_degree3_slots(const qldpc_bp *bp, int32_t *d3k);

/* Min-sum decoder on engine 6 (bp_hbm.hip): messages in HBM as coalesced
 * [edge][lane] arrays, one decode per lane, waves independent.  The engine every
 * create call falls back to when no LDS engine holds a decode's image (> 160
 * KiB: e.g. the fp64 space-time graph of hgp_34_n1225_q3 at num_rep 3) or a
 * column degree exceeds 8; this entry point forces it for any graph (row and
 * column degree <= 12: the compile-time edge blocks kHRow / kHCol of bp_hbm.hip;
 * larger degrees return QLDPC_ENOTSUP).  Same decode contract as qldpc_bp_create (the ldpc
 * bp_decoder replacement, src/Decoders.py:80-84); min-sum only. */
int qldpc_bp_create_hbm(qldpc_graph *g, const double *channel_probs, int32_t max_iter, double ms_scaling_factor,
                        int32_t precision, qldpc_bp **out);

/* BP+OSD in the fused shot loop (bposd_decoder per sector, src/Decoders.py:26-41, inside
 * _single_run, src/Simulators.py:117-168): after qldpc_mc_set_osd, qldpc_mc_launch captures
 * every decode that reaches max_iter (its last-iteration posteriors, syndrome and sampled
 * error) on the device, runs the GPU OSD stage (qldpc_osd_gpu) on those, re-checks their
 * residual against H and the logicals, and corrects the per-shot fail flags and the failure
 * counters -- no host copies beyond the per-sector candidate counts.  Engine-3 MC handles
 * only; each OSD handle must be built on its sector decoder's graph (NULL = plain BP).
 * With an OSD handle set, qldpc_mc_launch is SYNCHRONOUS on its stream (it reads the
 * candidate counts back to size the OSD launch).  Capture memory per sector is bounded by
 * QLDPC_OSD_CAPTURE_MB (default 2048; n*11 + m + 8 bytes per slot); a launch with more shots
 * than slots runs as consecutive pieces, so no candidate is ever dropped. */
int qldpc_mc_set_osd(qldpc_mc *mc, qldpc_osd_gpu *osd_x, qldpc_osd_gpu *osd_z);

/* Engine 3: extra LDS cycles of one variable-phase pass's CS gathers (summed
 * over gather instructions and lane groups: distinct checks on one bank beyond
 * the first) with the identity check order (`before`) and with the labels the
 * decoder uses (`after`, host-side label search at create time; QLDPC_LABEL=0
 * disables it).  0 / 0 for the other engines. */
/* Static LDS model of the engine-3 fp64 variable phase, per workgroup and iteration (zeros for other
 * families): out6 = {CS-gather LDS cycles, of which bank-conflict extra; V-slot read cycles, extra;
 * v2c store group-cycles, extra} under the lane-group rules of MI355X_MICROARCH.md §LDS. */
int qldpc_bp_lds_model(const qldpc_bp *bp, int64_t *out6);
/* The same model for the fp64 m2s family's V-slot placement of graph g, host only (no device, no
 * decoder): the engine's geometry, degree sort, greedy placement and `anneal_iters` annealing moves
 * (< 0 = the default, 4000 per edge; 0 = greedy only).  ENOTSUP outside the m2s envelope. */
int qldpc_m2s_place_model(const qldpc_graph *g, int32_t anneal_iters, int64_t *out6);
int qldpc_bp_bank_stats(const qldpc_bp *bp, int32_t *before, int32_t *after);

/*
 * Multi-GPU.  Shots shard by global index with no data-path
 * exchange; the one collective is the sum of the int64 qldpc_counters vector,
 * which replaces the reference's fork-pool reduction (`parmap` + `np.sum`,
 * src/Simulators.py:37-61 and :170-188).  RCCL (over xGMI) is loaded at first use
 * (dlopen librccl.so.1); without it these return QLDPC_ENOTSUP.
 *   qldpc_comm_unique_id / qldpc_comm_init_rank : one process per GPU (rank 0
 *       makes the id, the host side ships its 128 bytes to every rank);
 *   qldpc_comm_init_all : one process driving ndev GPUs (devices NULL = 0..ndev-1),
 *       out = array of ndev handles;
 *   qldpc_comm_allreduce_counters : in-place sum of a device qldpc_counters on
 *       `stream` (async);
 *   qldpc_comm_allreduce_counters_group : the same for the handles of one
 *       process (qldpc_comm_init_all), one RCCL group call.
 */
#define QLDPC_COMM_ID_BYTES 128
typedef struct qldpc_comm qldpc_comm;
int qldpc_comm_unique_id(uint8_t *id_out);
int qldpc_comm_init_rank(int device, int32_t nranks, int32_t rank, const uint8_t *id, qldpc_comm **out);
int qldpc_comm_init_all(int32_t ndev, const int32_t *devices, qldpc_comm **out);
int qldpc_comm_rank(const qldpc_comm *comm, int32_t *rank, int32_t *nranks, int32_t *device);
int qldpc_comm_allreduce_counters(qldpc_comm *comm, void *d_counters, void *stream);
int qldpc_comm_allreduce_counters_group(qldpc_comm **comms, void **d_counters, void **streams, int32_t n);
int qldpc_comm_destroy(qldpc_comm *comm);

/*
 * `WordErrorRate(num_run)` over several GPUs from ONE host thread
 * (CodeSimulator_DataError.WordErrorRate, src/Simulators.py:170-188, whose
 * `parmap` fans shots out over CPU cores): MC handle d (one per device, each on
 * its own device's decoders) runs a contiguous block of the global shots (block
 * sizes S/ndev or S/ndev + 1, the first S%ndev devices one longer: the split of
 * parallel.shard_range), the counters are summed
 * with one grouped all-reduce (comms from qldpc_comm_init_all, in the same
 * device order: comms[d] must be rank d of ndev, on MC handle d's device, else
 * QLDPC_EINVAL; per-process qldpc_comm_init_rank communicators are refused) or,
 * with comms NULL, on the host; the sum is added to *out.  Each device is
 * driven from its own host thread (BP+OSD launches are synchronous).
 * Synchronous.  The ndev > 1 RCCL path has not yet run on a multi-GPU node.
 * Shots keyed by global index: the totals do not depend on ndev.
 */
/* The shot-block split qldpc_mc_run_sharded uses (= parallel.shard_range): part `part` of `nparts`
 * owns [begin, begin + count) of `total` shots, block sizes differ by <= 1, the first total % nparts
 * parts one longer.  Host-only (no GPU needed). */
int qldpc_shard_range(int64_t total, int32_t nparts, int32_t part, int64_t *begin, int64_t *count);
int qldpc_mc_run_sharded(qldpc_mc **mcs, qldpc_comm **comms, int32_t ndev, double px, double py, double pz,
                         uint64_t seed, uint64_t shot_begin, int64_t shot_count, int32_t logical_mode,
                         qldpc_counters *out);

/*
 * Circuit-level space-time shot loop (CodeSimulator_Circuit_SpaceTime._single_run / WordErrorRate,
 * src/Simulators_SpaceTime.py:968-1049) for many samples per launch.  Inputs (host CSR graphs
 * from qldpc_graph_create; qldpc_fault_tolerance_amd/circuit.py builds them):
 *   dem, dem_obs : detectors x mechanisms / observables x mechanisms of the FULL circuit's DEM
 *                  (the stim detector_sampler's distribution, :940; rows = num_cycles * m
 *                  detectors, num_cycles = num_rounds * num_rep + 1), probs [M] host doubles;
 *   dec1         : decoder1 on h1 (num_rep * m rows; GenFaultHyperGraph's first layer, :955);
 *   h1_space_cor : GenCorrecHyperGraph (m x n1), L1 (K x n1) the first layer's observables;
 *   dec2, L2     : decoder2 on h2 (m x n2) and the last layer's observables.
 * Sample s draws mechanism j when Philox4x32-10(key = seed, ctr = (j, shot, 0x51D50003)) as a
 * 53-bit uniform is < probs[j] (shot = shot_begin + s).  Counters: shots, failures, sector 0 =
 * decoder1 decodes (num_rounds per sample), sector 1 = decoder2 decodes.  d_fail [S] (or NULL),
 * d_detobs [S][D + K] sampled detector and observable bits (or NULL).  Asynchronous on `stream`
 * (no host round trip, BP+OSD included, unless the OSD is a host stage past the GPU envelope).  dec1 = dec2 = NULL (and NULL h1_space_cor / L1 /
 * L2) makes a sampler-only handle for qldpc_circ_sample (decoders outside the engine).
 */
typedef struct qldpc_circ qldpc_circ;
int qldpc_circ_create(const qldpc_graph *dem, const qldpc_graph *dem_obs, const double *probs, qldpc_bp *dec1,
                      const qldpc_graph *h1_space_cor, const qldpc_graph *L1, qldpc_bp *dec2, const qldpc_graph *L2,
                      int32_t num_rounds, int32_t num_rep, int64_t max_batch, qldpc_circ **out);
/* decoder2 as bposd_decoder (ST_BPOSD_Decoder_Circuit, src/Decoders_SpaceTime.py:277-292): dec2 from
 * qldpc_bp_create_soft and ONE of a GPU OSD or a host OSD stage on h2; a host stage is turned into a
 * GPU OSD with its method, order, rank and soft weights, so the launch never leaves the device —
 * except past the GPU kernel's envelope (n > 8192, osd_e order > 24), where the host stage decodes
 * the final layer (one synchronous D2H / H2D round trip per batch inside qldpc_circ_launch). */
int qldpc_circ_set_final_osd(qldpc_circ *circ, qldpc_osd_gpu *osd_gpu, const qldpc_osd *osd_host);
/* DEM sampler of qldpc_circ_launch / qldpc_circ_sample (stim's compile_detector_sampler().sample,
 * src/Simulators_SpaceTime.py:940, :1029): 1 = geometric skip (the default since round 6: per
 * mechanism and global 64-sample word, Philox-drawn gaps u < ceil(2^53 (1 - p)^k); ~1 + 64 p draws
 * per word), 0 = keyed (one Philox uniform per (sample, mechanism), u < p).  Both are exact
 * Bernoulli(p_j) samplers keyed by global sample indices (shard-invariant); they draw different
 * samples. */
int qldpc_circ_set_sampler(qldpc_circ *circ, int32_t sampler);
int qldpc_circ_info(const qldpc_circ *circ, int32_t *detectors, int32_t *observables, int32_t *mechanisms);
int qldpc_circ_launch(qldpc_circ *circ, uint64_t seed, uint64_t shot_begin, int64_t shot_count, void *d_counters,
                      uint8_t *d_fail, uint8_t *d_detobs, void *stream);
/* The sampling step alone (stim's detector sampler): d_out [S][D + K] uint8 detector then
 * observable bits of samples shot_begin.. (the draws qldpc_circ_launch decodes).  Async. */
int qldpc_circ_sample(qldpc_circ *circ, uint64_t seed, uint64_t shot_begin, int64_t shot_count, uint8_t *d_out,
                      void *stream);
int qldpc_circ_destroy(qldpc_circ *circ);

/*
 * The sampling step alone (CodeSimulator_DataError._generate_error,
 * src/Simulators.py:89-115): d_err uint8 [S][n], bit0 = x, bit1 = z, from the
 * Philox stream of qldpc_mc_launch (shot shot_begin + s, qubit j) or from
 * d_uniforms [S][n] (CPython's random() values) with the reference's 3-way
 * split.  Bit-identical to the d_err output of qldpc_mc_launch.  Async.
 */
int qldpc_sample_errors(double px, double py, double pz, uint64_t seed, uint64_t shot_begin, int64_t shot_count,
                        int32_t n, const double *d_uniforms, uint8_t *d_err, void *stream);

/* hipStreamSynchronize(stream) for hosts without a HIP binding (NULL = legacy default stream). */
int qldpc_stream_sync(void *stream);

#ifdef __cplusplus
}
#endif
#endif /* QLDPC_HIP_H */
