/*
 * smcdet_hip.h — C ABI of the MI355X (gfx950) hot path of the smcdet SMC
 * star-detection sampler.  Plain pointers and sizes only; every buffer is a
 * caller-owned, contiguous, float32 (unless stated) device allocation on the
 * device that owns `stream`.  Every entry point is asynchronous on `stream`
 * (a hipStream_t passed as void*), never allocates, never synchronises, and
 * returns 0 on success or a negative SMCDET_E* code; smcdet_last_error()
 * then describes the failure (thread-local).
 *
 * Layout follows the reference (timwhite0/smcdet): tiles lead, then
 * particles, then sources.  T = numH*numW tiles (row-major), N particles per
 * tile, S sources per particle (= Prior.max_objects), tile H x W pixels.
 *   tiled_image [T,H,W]   locs [T,N,S,2] (row h, column w)   fluxes [T,N,S]
 *   counts [T,N] (float32, as the reference)                  per-tile [T]
 *
 * Each entry point cites the reference interface it replaces.  The
 * reference has no FFI: its "plugin" boundary is duck-typed Python objects
 * (smcdet/sampler.py:10-37); the Python package smcdet_amd keeps those
 * classes and calls this ABI through ctypes.
 */
#ifndef SMCDET_HIP_H
#define SMCDET_HIP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define SMCDET_ABI_VERSION 18

/* status codes */
#define SMCDET_OK 0
#define SMCDET_EINVAL -1      /* bad argument (null pointer, size, enum) */
#define SMCDET_EUNSUPPORTED -2 /* shape outside what the kernels support */
#define SMCDET_EHIP -3        /* HIP runtime error (launch/config) */

/* image models */
#define SMCDET_MODEL_M71 1     /* M71ImageModel: 3-component PSF, Gaussian noise */
#define SMCDET_MODEL_POISSON 2 /* ImageModel: Normal-pdf PSF, Poisson noise      */

/* priors */
#define SMCDET_PRIOR_M71 1    /* M71Prior: Poisson count, uniform locs, truncated-Pareto flux */
#define SMCDET_PRIOR_PARETO 2 /* ParetoStarPrior: uniform count, uniform locs, Pareto flux   */

/* resampling */
#define SMCDET_RESAMPLE_MULTINOMIAL 0
#define SMCDET_RESAMPLE_SYSTEMATIC 1

/* mh flags */
#define SMCDET_MH_FULL_RECOMPUTE 1u /* re-render every source per step (reference arithmetic) */
/* draw the moved component from 0..count-1 instead of 0..S-1: a particle of
 * count s padded to S sources then moves exactly as the reference's
 * fixed-count kernel with S = s (kernel.py:35-37); count 0 never moves.
 * Used by the count-stratified sampler (CS-SMC). */
#define SMCDET_MH_COMPONENT_BY_COUNT 2u
/* independent stopping: tiles whose temperature is already 1 are not mutated
 * (their particles are only gathered through `ancestors`) */
#define SMCDET_MH_SKIP_DONE 4u

/* (no flag) A location proposal clamped onto the prior box's upper edge
 * (distributions.py:48) has log prior -inf (Uniform.log_prob(high),
 * prior.py:73) and is rejected; as in the reference, whose cached log target
 * then becomes -inf * 0 = NaN (kernel.py:125), the particle also rejects every
 * remaining proposal of that sweep. */

/* temper_reweight flags */
/* independent stopping: a tile that entered at temperature 1 keeps it (delta
 * 0), gets uniform weights, an unchanged log Z and ESS (that of its last
 * step) and identity resampling indices, so its final particles stay put
 * while the other tiles run on.
 * Without it (the reference, sampler.py:230) such tiles are resampled and
 * mutated at temperature 1 until every tile has finished. */
#define SMCDET_SMC_FREEZE_DONE 1u
/* smcdet_mh_sweep_step only: run the tile pass as its own launch right after
 * the sweep even where the shape could fuse (same results).  The default in
 * SMCsampler: on gfx950 the separate 512-thread tile kernel (~27 us at
 * N = 4096) beats the fused tail on the sweep's 256-thread workgroup (~30 us),
 * and back-to-back launches on one stream leave no gap to recover
 * (DESIGN.md §4.2). */
#define SMCDET_SMC_TWO_LAUNCH 2u
/* Flags marked "diagnostic build only" are compiled into
 * libsmcdet_hip_diag.so (make diag, -DSMCDET_DIAG) alone: the product library
 * returns SMCDET_EUNSUPPORTED for them before any device work.
 * diagnostic build only: ablations (timing only; results are NOT valid samples) */
#define SMCDET_MH_ABLATE_LIKELIHOOD 256u /* skip the delta-likelihood passes */
#define SMCDET_MH_ABLATE_PROPOSAL 512u   /* skip the truncated-normal proposal math */
/* diagnostic build only: evaluate the union window one position per lane instead of two
 * (packed arithmetic); same results up to float32 summation order */
#define SMCDET_MH_SCALAR_SLOTS 1024u
/* diagnostic: small tiles (H*W <= 64) without the per-wave PSF cache (the
 * moved source's old PSF re-evaluated each iteration); same results */
#define SMCDET_MH_NO_PSF_CACHE 2048u
/* diagnostic build only: M71 tiles of 65..1024 pixels without the per-wave 1/v image
 * (each pixel's 1/(s0^2 + eta*rate) formed per use); same results */
#define SMCDET_MH_NO_RCP_CACHE 4096u
/* diagnostic build only: M71 sweeps with the radial PSF table in LDS (the union
 * window's PSF values from a cubic table instead of exp2/log2; results differ
 * by float32 rounding of the profile, ~3e-7 relative).  Measured slower at
 * 32x32 (its LDS reads) and even at 8x8, so off by default */
#define SMCDET_MH_PSF_TABLE 8192u
/* diagnostic: M71 tiles of 16x16 .. 1024 pixels without the block form of
 * same-anchor steps (the union window's first 16 rows and columns as one
 * 16x16 block whose Gaussian PSF terms come from a rank-4 MFMA); results
 * differ by float32 rounding of the profile */
#define SMCDET_MH_NO_BLOCK 16384u

/* Image model (smcdet/images.py:6-26 ImageModel, :105-145 M71ImageModel). */
typedef struct smcdet_image_model {
  int32_t model;          /* SMCDET_MODEL_* */
  int32_t H, W;           /* tile height / width in pixels */
  int32_t psf_radius;     /* R: (2R+1)^2 window anchored at floor(loc) */
  float background;       /* additive background (ADU) */
  float adu_per_nmgy;     /* M71 flux scale; 1 for POISSON */
  float psf_params[6];    /* M71: sigma1, sigma2, sigmap, beta, b, p0; POISSON: [0]=psf_stdev */
  float psf_norm;         /* M71 normalising constant C (images.py:122-135) */
  float noise_additive;   /* M71: variance = noise_additive + noise_multiplicative*rate */
  float noise_multiplicative;
} smcdet_image_model_t;

/* Prior (smcdet/prior.py:8-75, :78-101, :157-189, :192-226). */
typedef struct smcdet_prior {
  int32_t kind;           /* SMCDET_PRIOR_* */
  int32_t min_objects, max_objects;
  float loc_low;          /* -pad */
  float loc_high_h;       /* H + pad */
  float loc_high_w;       /* W + pad */
  float poisson_mean;     /* M71: counts_rate*(H+2pad)*(W+2pad) */
  float flux_alpha;
  float flux_lower;       /* M71: truncated-Pareto lower; PARETO: flux_scale */
  float flux_upper;       /* M71: truncated-Pareto upper; PARETO: unused */
} smcdet_prior_t;

/* Single-component MH kernel (smcdet/kernel.py:7-24). */
typedef struct smcdet_mh {
  int32_t num_iters;
  float locs_stdev;
  float fluxes_stdev;
  float fluxes_min, fluxes_max;
  float locs_min_h, locs_min_w; /* = Prior.loc_prior.low  (sampler.py:36) */
  float locs_max_h, locs_max_w; /* = Prior.loc_prior.high (sampler.py:37) */
} smcdet_mh_t;

/* Optional replay of recorded draws (tests): per MH iteration k, tile t,
 * particle n: the chosen component, the two location uniforms and the flux
 * uniform of the chosen component, and the accept uniform.
 * trace_loga / trace_accept (nullable; smcdet_mh_sweep / _step only): the
 * sweep writes each decision's log alpha (float32, as the kernel evaluated
 * it) and its accept flag (0/1) at [k,t,n] -- decision-by-decision parity
 * against recorded reference decisions (kernel.py:114-116).  Iterations a
 * particle does not run (after an upper-edge freeze, or K = 0) are left
 * untouched.  Only the replay instantiation carries these stores. */
typedef struct smcdet_mh_replay {
  const int32_t* comp; /* [K,T,N]   */
  const float* uloc;   /* [K,T,N,2] */
  const float* uflux;  /* [K,T,N]   */
  const float* uacc;   /* [K,T,N]   */
  float* trace_loga;   /* [K,T,N] (nullable) */
  uint8_t* trace_accept; /* [K,T,N] (nullable) */
} smcdet_mh_replay_t;

/* "smcdet_hip <version> (gfx950) src <sha1 of the library's sources>" */
const char* smcdet_version(void);
int32_t smcdet_abi_version(void);
const char* smcdet_last_error(void);

/* Pinned, device-mapped host memory (hipHostMalloc): *host is the host
 * address, *device the address kernels use; zero-filled.  For small
 * device->host signals without a copy launch (smcdet_temper_reweight's
 * live_host).  Free with smcdet_host_free(host). */
int smcdet_host_alloc(size_t bytes, void** host, void** device);
int smcdet_host_free(void* host);

/* Per-launch kernel timing for benchmarks (no reference counterpart).  While
 * enabled, each of the next max_launches sweep launches (smcdet_mh_sweep,
 * smcdet_mh_sweep_step, smcdet_mala_sweep) is dispatched by
 * hipExtLaunchKernel with a start/stop event pair of an internal pool: the
 * events are stamped by the kernel's own dispatch, so timing adds no marker
 * packet (and no launch bubble) between kernels.  max_launches = 0 disables
 * timing and frees the pool; a new call discards earlier timings.
 * smcdet_launch_timing_read waits for the timed launches and writes the first
 * min(max, *n_out) durations in ms; *n_out = launches timed since enabling.
 * The pool is process-global and not thread-safe: enable, launch and read
 * from one host thread (bench.py does). */
int smcdet_launch_timing(int32_t max_launches);
int smcdet_launch_timing_read(float* ms, int32_t max, int32_t* n_out);
/* The same launches' start times in ms after the first timed launch's start
 * (launch-to-launch intervals: the step-time spread bench.py reports). */
int smcdet_launch_timing_starts(float* ms, int32_t max, int32_t* n_out);
/* on != 0: while timing is enabled, the per-tile temper / reweight /
 * resampling launches (smcdet_temper, smcdet_update_weights,
 * smcdet_temper_reweight and the tile pass of a two-launch
 * smcdet_mh_sweep_step) also take event pairs from the pool, in launch order
 * with the sweeps (a two-launch SMC step: sweep, then tile pass).  Off by
 * default; smcdet_launch_timing(0) turns it off. */
int smcdet_launch_timing_tiles(int32_t on);

/* ImageModel.loglikelihood / M71ImageModel.loglikelihood
 * (smcdet/images.py:85-102, :159-175): out[T,N].  Tiles up to 4096 pixels
 * (either model) stage the tile in LDS; M71 tiles up to 65536 pixels render
 * 64-pixel chunks in registers and read the tile from global memory
 * (smcdet_render likewise).  MALA, MCMC chains and aggregation sweeps keep
 * the 4096-pixel LDS budget. */
int smcdet_loglik(const smcdet_image_model_t* model, const float* tiled_image,
                  const float* locs, const float* fluxes, int32_t T, int32_t N,
                  int32_t S, float* out, void* stream);

/* rate image lambda = B + sum_j g*f_j*psf_j  (images.py:80-82, :149-154):
 * rate[T,H,W,N] (the layout the reference's ImageModel.sample produces). */
int smcdet_render(const smcdet_image_model_t* model, const float* locs,
                  const float* fluxes, int32_t T, int32_t N, int32_t S,
                  float* rate, void* stream);

/* ImageModel.psf (smcdet/images.py:28-76): dense psf[T,H,W,N,S]. */
int smcdet_psf_dense(const smcdet_image_model_t* model, const float* locs,
                     int32_t T, int32_t N, int32_t S, float* psf, void* stream);

/* Noise draw for ImageModel.sample (images.py:78-83 Poisson, :147-157
 * Normal): image[T,H,W,N] from rate[T,H,W,N] (in place allowed). */
int smcdet_sample_image(const smcdet_image_model_t* model, const float* rate,
                        int64_t count, uint64_t seed, uint64_t offset,
                        float* image, void* stream);

/* Per-tile location boxes (every function taking `tile_boxes`): a nullable
 * [T,4] float array (lo_h, lo_w, hi_h, hi_w) that replaces the prior's
 * [-pad, H+pad) x [-pad, W+pad) for tile t -- the tiles' boxes then partition
 * the padded image (padding only on its outer edges), so the product of the
 * tiles' priors is the whole image's prior (used by tile aggregation,
 * DESIGN.md §9).  An M71 prior's Poisson count mean scales with the box
 * area.  Null: the reference's per-tile padding (prior.py:17-23). */

/* Prior.log_prob (smcdet/prior.py:67-75, :183-189, :220-226): out[T,N]. */
int smcdet_log_prior(const smcdet_prior_t* prior, const float* counts,
                     const float* locs, const float* fluxes, int32_t T,
                     int32_t N, int32_t S, const float* tile_boxes, float* out,
                     void* stream);

/* Prior.sample(stratify_by_count=True, num_catalogs_per_count=n_per_count)
 * (smcdet/prior.py:25-64, :201-217): N = (max-min+1)*n_per_count.
 * uloc [T,N,S,2] / uflux [T,N,S] replay the uniforms when non-null. */
int smcdet_prior_sample(const smcdet_prior_t* prior, int32_t T,
                        int32_t n_per_count, uint64_t seed, uint64_t offset,
                        const float* uloc, const float* uflux,
                        const float* tile_boxes, float* counts, float* locs,
                        float* fluxes, void* stream);

/* SingleComponentMH.run (smcdet/kernel.py:26-130), K = mh->num_iters
 * iterations fused in one launch.  Reads the state of particle
 * ancestors[t,n] (identity when null) from *_in and writes the mutated
 * state to *_out (in place allowed when ancestors is null).  counts_out may
 * be null.  temperature[T].  Outputs: acc_rate[T] = acceptance rate of the
 * LAST iteration (kernel.py:130); loglik_out[T,N] (nullable) = the image
 * log-likelihood of the returned state (what SMCsampler.temper recomputes,
 * sampler.py:100-102).  acc_count[2T] is an int32 workspace, 8-byte aligned,
 * that must be zero before the first call; every call leaves it zero again
 * (it holds the per-tile accept counters and workgroup tickets only while the
 * kernel runs), so one zeroed buffer serves every call on a stream.
 * rate_in / rate_out [T,N,H*W] (both nullable, ignored with
 * SMCDET_MH_FULL_RECOMPUTE): persisted per-particle rate images
 * lambda = B + sum_j g f_j psf_j.  With rate_in the sweep starts from the
 * image of particle ancestors[t,n] instead of re-rendering all S sources;
 * rate_out receives the image of the returned state (maintained
 * incrementally, float32 update rounding).  rate_in must describe *_in
 * exactly; rate_in != rate_out when ancestors is non-null.
 * Tiles above 4096 pixels (M71 model, up to 65536 = 256x256 pixels): the tile
 * image and the rate images live in global memory -- rate_in / rate_out are
 * [T,N,H*W+64] (64 dummy cells per row for masked lanes), rate_out is
 * REQUIRED (the sweep updates its rows in place; with FULL_RECOMPUTE their
 * contents afterwards are unspecified), rate_in == rate_out is allowed
 * without ancestors, and the fused step (smcdet_mh_sweep_step) runs as two
 * launches.
 * go (nullable, int32 device scalar): when *go == 0 the launch does nothing
 * (no output is written) -- lets a host enqueue the next SMC iteration before
 * it has read the loop condition (see smcdet_temper_reweight's `live`).
 * tile_boxes (nullable): per-tile location boxes in place of mh->locs_min/max. */
int smcdet_mh_sweep(const smcdet_image_model_t* model,
                    const smcdet_prior_t* prior, const smcdet_mh_t* mh,
                    const float* tiled_image, const float* temperature,
                    int32_t T, int32_t N, int32_t S, const int64_t* ancestors,
                    const float* counts_in, const float* locs_in,
                    const float* fluxes_in, float* counts_out,
                    float* locs_out, float* fluxes_out, const float* rate_in,
                    float* rate_out, uint64_t seed,
                    uint64_t offset, const smcdet_mh_replay_t* replay,
                    uint32_t flags, float* loglik_out, float* acc_rate,
                    int32_t* acc_count, const int32_t* go,
                    const float* tile_boxes, void* stream);

/* SingleComponentMALA.run (smcdet/kernel.py:133-275), K iterations fused in
 * one launch.  Arguments as smcdet_mh_sweep; mala->locs_stdev and
 * mala->fluxes_stdev carry the step sizes (locs_step, fluxes_step,
 * kernel.py:134-145).  The gradient of log_target w.r.t. the chosen source's
 * (h, w, f) -- what torch.autograd.grad computes (kernel.py:160-166,
 * :190-197) -- is evaluated analytically in-kernel over the source's PSF
 * window.  Flags: SMCDET_MH_COMPONENT_BY_COUNT, SMCDET_MH_SKIP_DONE.
 * The replay layout is smcdet_mh_replay_t's; `go` as smcdet_mh_sweep. */
int smcdet_mala_sweep(const smcdet_image_model_t* model,
                      const smcdet_prior_t* prior, const smcdet_mh_t* mala,
                      const float* tiled_image, const float* temperature,
                      int32_t T, int32_t N, int32_t S, const int64_t* ancestors,
                      const float* counts_in, const float* locs_in,
                      const float* fluxes_in, float* counts_out,
                      float* locs_out, float* fluxes_out, const float* rate_in,
                      float* rate_out, uint64_t seed,
                      uint64_t offset, const smcdet_mh_replay_t* replay,
                      uint32_t flags, float* loglik_out, float* acc_rate,
                      int32_t* acc_count, const int32_t* go, void* stream);

/* MHsampler.run (smcdet/sampler.py:301-486): one single-component MH chain
 * per (tile, chain) at temperature 1 -- C chains per tile, T tiles (the
 * reference runs C = 1).  locs_state [T,C,S,2] / fluxes_state [T,C,S] hold
 * the chain state (the initial sample on the first call) and are updated in
 * place; iterations [k_begin, k_end) of num_samples_total - 1 run in this
 * call (chunked runs continue the same Philox streams).  Sample m is the
 * state after iteration m-1 (sample 0 = the initial state); samples
 * m >= num_samples_burnin with (m - burnin) % keep_every_k == 0 are written to
 * locs_out [T,C,M,S,2] / fluxes_out [T,C,M,S], M = ceil((total - burnin) /
 * keep), the reference's burn_thin_idx (sampler.py:339-341).  accept_out
 * [T,C,total-1] int32 (nullable): the accept flag of every iteration.
 * mh->locs_stdev / fluxes_stdev / bounds as in smcdet_mh_sweep (the
 * reference takes the flux bounds from Prior.flux_lower/flux_upper).  Replay
 * buffers: comp [total-1,T,C], uloc [total-1,T,C,2], uflux / uacc
 * [total-1,T,C].  frozen [T,C] int32 (nullable, zero before the first call):
 * a chain whose location proposal lands on the prior box's upper edge
 * rejects it and every later proposal of the run, as the reference's NaN
 * cached target does (sampler.py:522-526); the flag carries that across
 * chunked calls. */
int smcdet_mh_chain(const smcdet_image_model_t* model,
                    const smcdet_prior_t* prior, const smcdet_mh_t* mh,
                    const float* tiled_image, int32_t T, int32_t C, int32_t S,
                    const float* counts, float* locs_state, float* fluxes_state,
                    int32_t num_samples_total, int32_t num_samples_burnin,
                    int32_t keep_every_k, int32_t k_begin, int32_t k_end,
                    uint64_t seed, uint64_t offset,
                    const smcdet_mh_replay_t* replay, float* locs_out,
                    float* fluxes_out, int32_t* accept_out, int32_t* frozen,
                    void* stream);

/* SMCsampler.temper (smcdet/sampler.py:93-125) on device: per tile, delta
 * solves exp(2 LSE(delta*l) - LSE(2 delta*l)) = ess_threshold on (0, 1-tau]
 * (or delta = 1-tau when the ESS there is still above threshold).
 * temperature[T] is updated in place (float32 tau + delta); temperature_prev
 * receives the old value. */
int smcdet_temper(const float* loglik, float* temperature,
                  float* temperature_prev, int32_t T, int32_t N,
                  double ess_threshold, void* stream);

/* SMCsampler.update_weights (smcdet/sampler.py:181-196). */
int smcdet_update_weights(const float* loglik, const float* temperature,
                          const float* temperature_prev,
                          float* log_weights_unnorm, float* weights,
                          float* ess, float* log_norm_const, int32_t T,
                          int32_t N, void* stream);

/* Resampling indices (smcdet/sampler.py:127-150): systematic
 * (bucketize of (n+U)/N into cumsum(W)) or multinomial (iid).  u replays the
 * uniforms when non-null ([T] systematic, [T,N] multinomial). */
int smcdet_resample_index(const float* weights, int32_t T, int32_t N,
                          int32_t method, uint64_t seed, uint64_t offset,
                          const float* u, int64_t* idx, void* stream);

/* temper + update_weights (+ resample index when idx != null) fused: one
 * launch per SMC iteration instead of three.  flags: SMCDET_SMC_*.
 * finished_iter [T] (nullable, int32): set to `iter` when a tile's
 * temperature reaches 1 while it holds a negative value (per-tile finishing
 * iteration).  live [3] (nullable, int32, 8-byte aligned, zero before the first call): after
 * the call live[2] = the number of tiles still below temperature 1 (the
 * reference's while condition, sampler.py:230); live[0..1] are workspace and
 * left zero.  go (nullable): when *go == 0 the launch does nothing.
 * live_host (nullable, used with live): pinned, device-accessible host memory
 * (hipHostMalloc) that also receives live[2], so a host can read the count
 * once the launch has completed without enqueueing a copy. */
int smcdet_temper_reweight(const float* loglik, float* temperature,
                           float* temperature_prev, float* log_weights_unnorm,
                           float* weights, float* ess, float* log_norm_const,
                           int32_t T, int32_t N, double ess_threshold,
                           int32_t resample_method, uint64_t seed,
                           uint64_t offset, int64_t* idx, uint32_t flags,
                           int32_t* finished_iter, int32_t iter, int32_t* live,
                           const int32_t* go, int32_t* live_host, void* stream);

/* The temper / reweight / resample-index half of a fused SMC iteration
 * (smcdet_mh_sweep_step): the arguments of smcdet_temper_reweight that the
 * sweep does not already carry (its loglik_out and temperature are the
 * pass's log-likelihoods and temperatures).  resample_u [T] (nullable)
 * replays the systematic offsets (tests); multinomial draws are not
 * replayable here. */
typedef struct smcdet_smc_tail {
  float* temperature_prev;
  float* log_weights_unnorm;
  float* weights;
  float* ess;
  float* log_norm_const;
  double ess_threshold;
  int32_t resample_method;
  uint32_t flags;            /* SMCDET_SMC_* */
  uint64_t seed;
  uint64_t offset;
  int64_t* idx;              /* [T,N] next resampling indices (nullable) */
  const float* resample_u;   /* [T] systematic U replay (nullable) */
  int32_t* finished_iter;
  int32_t* live;
  int32_t* live_host;
  int32_t iter;
  int32_t reserved;
  /* (ABI 16) systematic resampling handed to the next sweep as bins instead
   * of indices: bins_out (nullable; SMCDET_BINS_FLOATS(T, N) floats) receives
   * the tile's running sum of the new weights, [T*N] (float32 roundings of the
   * float64 cumsum), then the T offsets U, then (ABI 17) per tile the 64
   * chunk-end bins of the search's first level, [T*64]: entry l is
   * bins[min((l+1)*c, N) - 1] for l < ceil(N/c), c = ceil(N/64) -- so the
   * first level reads 256 contiguous bytes per wave instead of 64 strided
   * lines.  The tile pass then skips the index search; anc_bins (nullable,
   * input) is such a buffer from the previous step, and each wave of this
   * sweep finds its own ancestor in it (idx[n] = #{i : bins[i] < (n + U)/N},
   * clamped to N - 1: the same indices, bit for bit) in place of
   * `ancestors`.  smcdet_bins_index converts a buffer to the indices. */
  const float* anc_bins;
  float* bins_out;
} smcdet_smc_tail_t;

/* One SMC iteration of SMCsampler.run (smcdet/sampler.py:221-237: resample
 * -> mutate -> temper -> update_weights, the resample being the sweep's
 * ancestor gather): smcdet_mh_sweep followed by smcdet_temper_reweight on its
 * loglik_out (required), with the same results bit for bit.  One launch: the
 * last workgroup to finish a tile runs the tile's temper / reweight / index
 * pass in the sweep's own LDS, so the pass starts the moment the tile's last
 * particle is done and the step pays one launch instead of two.  Shapes the
 * fused form does not cover (N % 4 != 0, N > 4096, tiles of <= 64 pixels,
 * SMCDET_MH_FULL_RECOMPUTE, an LDS budget that would cost occupancy) run as
 * the two launches; smcdet_mh_sweep_step_fused() reports which. */
int smcdet_mh_sweep_step(const smcdet_image_model_t* model,
                         const smcdet_prior_t* prior, const smcdet_mh_t* mh,
                         const float* tiled_image, float* temperature,
                         int32_t T, int32_t N, int32_t S,
                         const int64_t* ancestors, const float* counts_in,
                         const float* locs_in, const float* fluxes_in,
                         float* counts_out, float* locs_out, float* fluxes_out,
                         const float* rate_in, float* rate_out, uint64_t seed,
                         uint64_t offset, const smcdet_mh_replay_t* replay,
                         uint32_t flags, float* loglik_out, float* acc_rate,
                         int32_t* acc_count, const int32_t* go,
                         const float* tile_boxes, const smcdet_smc_tail_t* tail,
                         void* stream);
/* 1 when smcdet_mh_sweep_step runs these shapes as one launch, else 0. */
int smcdet_mh_sweep_step_fused(const smcdet_image_model_t* model, int32_t N,
                               int32_t S, uint32_t flags);

/* Gather of the resampled state (smcdet/sampler.py:150-169). */
/* The systematic resampling indices [T,N] of a bins buffer (the tail's
 * bins_out layout: [T*N] running sums, [T] offsets U, [T*64] first-level
 * chunk ends): idx[t,n] = #{i : bins[t,i] < (n + U_t)/N} clamped to N - 1
 * (sampler.py:141-148). */
#define SMCDET_BINS_FLOATS(T, N) ((size_t)(T) * (size_t)(N) + (size_t)(T) * 65u)
int smcdet_bins_index(const float* bins, int32_t T, int32_t N, int64_t* idx, void* stream);

int smcdet_gather(const int64_t* idx, int32_t T, int32_t N, int32_t S,
                  const float* counts_in, const float* locs_in,
                  const float* fluxes_in, float* counts_out, float* locs_out,
                  float* fluxes_out, void* stream);

/* Count-stratified SMC combination (manuscript/manuscript.tex:344-354,
 * Algorithm 2; the reference describes CS-SMC but has no code for it at HEAD).
 * Per image tile t, with NS count strata k (count s_min + k) whose fixed-count
 * samplers ran as "stratum tiles" t*NS + k of N equally weighted particles:
 *   probs[t,k] = p(s|x) = softmax_k(log_norm_const[t*NS+k] + log_count_prior[k])
 *   (log_count_prior [T,NS] per tile when lcp_per_tile != 0: tile boxes)
 *   then n_out catalogs: stratum k_n ~ probs[t,:] (systematic: u_n = (n+U)/n_out,
 *   first k with cumsum(probs) >= u_n; multinomial: iid u_n), and a uniform
 *   particle m_n = floor(v_n * N) of that stratum; idx[t,n] = k_n*N + m_n and
 *   the catalog (counts [T,NS,N], locs [T,NS,N,S,2], fluxes [T,NS,N,S]) is
 *   gathered to counts_out [T,n_out], locs_out, fluxes_out.
 * u_strata ([T] systematic / [T,n_out] multinomial) and u_pick [T,n_out]
 * replay the uniforms when non-null. */
int smcdet_count_posterior(const float* log_norm_const,
                           const float* log_count_prior, int32_t lcp_per_tile,
                           int32_t T, int32_t NS,
                           int32_t N, int32_t S, int32_t n_out,
                           int32_t resample_method, uint64_t seed,
                           uint64_t offset, const float* u_strata,
                           const float* u_pick, const float* counts_in,
                           const float* locs_in, const float* fluxes_in,
                           float* probs, int64_t* idx, float* counts_out,
                           float* locs_out, float* fluxes_out, void* stream);

/* SMCsampler.prune (smcdet/sampler.py:198-219): counts_out[T,N] int64,
 * kept sources compacted to the front in their original order. */
int smcdet_prune(const float* locs, const float* fluxes, int32_t T, int32_t N,
                 int32_t S, float tile_dim, float flux_threshold,
                 int64_t* counts_out, float* locs_out, float* fluxes_out,
                 void* stream);

/* ---- tile aggregation (smcdet/aggregate.py:8-593, Aggregate) ------------- */
#define SMCDET_AGG_MAX_SOURCES 4096

/* Aggregate.mutate (aggregate.py:176-187 with log_target :105-130): K =
 * mh->num_iters single-component MH iterations on joint tiles of
 * model->H x model->W pixels (T tiles, N particles, S source slots), under
 *   log p(z) + (1 - tau) * [l_c1(z_1) + l_c2(z_2)] + tau * l_p(z),
 * l_p the joint tile's image log-likelihood, l_c1 / l_c2 those of its two
 * halves along `axis` (0: h, 1: w), each rendered from the sources whose axis
 * coordinate is <= dim/2 (first half) or > dim/2 (second), the reference's
 * unjoin (aggregate.py:265-324).  The moved component is drawn from
 * 0..count-1 (slots past the count hold zero flux and never move); proposals,
 * accept rule and the upper-edge freeze as smcdet_mh_sweep.  Reads particle
 * ancestors[t,n] (identity when null) from *_in; counts_out nullable.
 * loglik_parent / loglik_children [T,N] (nullable): l_p and l_c1 + l_c2 of the
 * returned state, from a fresh render (num_iters = 0 evaluates the input
 * state).  acc_rate [T] (nullable) = acceptance rate of the last iteration,
 * with acc_count [2T] as in smcdet_mh_sweep.  Replay layout as
 * smcdet_mh_replay_t (comp must be < count).  tile_boxes (nullable): per
 * joint tile location boxes in place of mh->locs_min/max.
 * workspace (nullable): joint tiles whose image, two rate images and catalog
 * per wave do not fit LDS at 4 waves per workgroup (smcdet_aggregate_workspace
 * > 0; M71 model, up to 65536 pixels and 4096 sources) keep them in this
 * caller-owned device buffer of smcdet_aggregate_workspace() floats and read
 * the tile image from global memory. */
int smcdet_aggregate_sweep(const smcdet_image_model_t* model,
                           const smcdet_prior_t* prior, const smcdet_mh_t* mh,
                           int32_t axis, const float* tiled_image,
                           const float* temperature, int32_t T, int32_t N,
                           int32_t S, const int64_t* ancestors,
                           const float* counts_in, const float* locs_in,
                           const float* fluxes_in, float* counts_out,
                           float* locs_out, float* fluxes_out, uint64_t seed,
                           uint64_t offset, const smcdet_mh_replay_t* replay,
                           float* loglik_parent, float* loglik_children,
                           float* acc_rate, int32_t* acc_count,
                           const float* tile_boxes, float* workspace, void* stream);
/* Floats of workspace smcdet_aggregate_sweep needs for these shapes (0: the
 * LDS path runs; < 0: unsupported, smcdet_last_error says why). */
int64_t smcdet_aggregate_workspace(const smcdet_image_model_t* model, int32_t T,
                                   int32_t N, int32_t S);

/* Aggregate.temper (aggregate.py:140-174), per count group: the particles of
 * each joint tile are sorted by count and split into G segments (count
 * groups) given by seg_tile[g], seg_start[g] (first particle within the
 * tile) and seg_len[g] (device int32 arrays).  With l = loglik_parent -
 * loglik_children, delta[g] solves exp(2 LSE(delta*l) - LSE(2 delta*l)) =
 * ess_threshold_prop * seg_len[g] on (0, 1 - tau] (brentq, xtol = rtol =
 * 1e-6), or is 1 - tau when the ESS there is still above it. */
int smcdet_aggregate_temper(const float* loglik_parent,
                            const float* loglik_children,
                            const float* temperature, int32_t T, int32_t N,
                            int32_t G, const int32_t* seg_tile,
                            const int32_t* seg_start, const int32_t* seg_len,
                            double ess_threshold_prop, float* delta,
                            void* stream);

/* Aggregate.update_weights (aggregate.py:439-483) + resample_intracount
 * (:485-521) per count group, after the caller has set temperature[t] to
 * temperature_prev[t] + the minimum of the tile's delta[g] (aggregate.py:171-
 * 174).  Per segment: log_weights_unnorm = (temperature - temperature_prev) *
 * l (float32), weights_intracount = softmax within the segment,
 * log_norm_const[g] += log mean exp(log w) (in place), ess[g] = 1 / sum w^2.
 * idx [T,N] (nullable): tile-local multinomial resampling indices drawn within
 * each segment from its weights (u [T,N] replays the uniforms). */
int smcdet_aggregate_reweight(const float* loglik_parent,
                              const float* loglik_children,
                              const float* temperature,
                              const float* temperature_prev, int32_t T,
                              int32_t N, int32_t G, const int32_t* seg_tile,
                              const int32_t* seg_start, const int32_t* seg_len,
                              float* log_weights_unnorm,
                              float* weights_intracount, float* log_norm_const,
                              float* ess, uint64_t seed, uint64_t offset,
                              const float* u, int64_t* idx, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* SMCDET_HIP_H */
