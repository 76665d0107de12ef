// Host sanitizer driver for the C ABI (include/smcdet_hip.h): the library's
// host side compiled with -Xarch_host -fsanitize=address,undefined (device
// code not built: nothing is launched) by `make asan`, run by
// tests/test_sanitizers.py without a GPU.  Every entry point is called with
// the argument errors its validation must reject (null buffers, empty or
// oversized shapes, unknown enums, inconsistent flags) and must return the
// documented negative code with a message, touching no device memory.
#include <cstdio>
#include <cstring>

#include "../../include/smcdet_hip.h"

static int fails = 0;
#define EXPECT(expr, code)                                                         \
  do {                                                                             \
    const long long rc_ = (long long)(expr);                                       \
    if (rc_ != (code)) {                                                           \
      std::printf("FAIL %s -> %lld (want %d): %s\n", #expr, rc_, (code),           \
                  smcdet_last_error());                                            \
      ++fails;                                                                     \
    } else if (std::strlen(smcdet_last_error()) == 0 && (code) != 0) {             \
      std::printf("FAIL %s: empty error message\n", #expr);                       \
      ++fails;                                                                     \
    }                                                                              \
  } while (0)

int main() {
  std::printf("%s abi %d\n", smcdet_version(), smcdet_abi_version());
  if (smcdet_abi_version() != SMCDET_ABI_VERSION) ++fails;
  smcdet_image_model_t m{};
  m.model = SMCDET_MODEL_M71;
  m.H = m.W = 32;
  m.psf_radius = 8;
  m.background = 104.f;
  m.adu_per_nmgy = 241.f;
  float pp[6] = {1.1f, 2.1f, 2.3f, 5.2f, 0.73f, 0.51f};
  std::memcpy(m.psf_params, pp, sizeof pp);
  m.psf_norm = 12.75f;
  m.noise_additive = 1e-10f;
  m.noise_multiplicative = 1.94f;
  smcdet_prior_t p{};
  p.kind = SMCDET_PRIOR_M71;
  p.min_objects = p.max_objects = 10;
  p.loc_low = -4.f;
  p.loc_high_h = p.loc_high_w = 36.f;
  p.poisson_mean = 4.f;
  p.flux_alpha = 0.21f;
  p.flux_lower = 0.063f;
  p.flux_upper = 1804.f;
  smcdet_mh_t mh{};
  mh.num_iters = 10;
  mh.locs_stdev = 0.1f;
  mh.fluxes_stdev = 2.5f;
  float dummy[16] = {0};
  float* d = dummy;
  alignas(8) int32_t ws[4] = {0};

  EXPECT(smcdet_loglik(nullptr, d, d, d, 1, 1, 1, d, nullptr), SMCDET_EINVAL);
  EXPECT(smcdet_loglik(&m, nullptr, d, d, 1, 1, 1, d, nullptr), SMCDET_EINVAL);
  EXPECT(smcdet_loglik(&m, d, d, d, 0, 1, 1, d, nullptr), SMCDET_EUNSUPPORTED);
  EXPECT(smcdet_loglik(&m, d, d, d, 70000, 1, 1, d, nullptr), SMCDET_EUNSUPPORTED);
  smcdet_image_model_t big = m;
  big.H = big.W = 300;
  EXPECT(smcdet_loglik(&big, d, d, d, 1, 1, 1, d, nullptr), SMCDET_EUNSUPPORTED);
  big.H = big.W = 100;
  big.model = SMCDET_MODEL_POISSON;
  EXPECT(smcdet_render(&big, d, d, 1, 1, 1, d, nullptr), SMCDET_EUNSUPPORTED);
  big.model = 7;
  EXPECT(smcdet_psf_dense(&big, d, 1, 1, 1, d, nullptr), SMCDET_EINVAL);
  EXPECT(smcdet_sample_image(&m, nullptr, 4, 0, 0, d, nullptr), SMCDET_EINVAL);
  EXPECT(smcdet_log_prior(nullptr, d, d, d, 1, 1, 1, nullptr, d, nullptr), SMCDET_EINVAL);
  smcdet_prior_t bp = p;
  bp.max_objects = 2;  // < min
  EXPECT(smcdet_log_prior(&bp, d, d, d, 1, 1, 1, nullptr, d, nullptr), SMCDET_EUNSUPPORTED);
  EXPECT(smcdet_prior_sample(&p, 1, 4, 0, 0, d, nullptr, nullptr, d, d, d, nullptr),
         SMCDET_EINVAL);
  // MH sweep: null buffers, S out of range, ancestors with aliased buffers,
  // negative K, zero proposal scale, incomplete replay, large tile without rate_out
  EXPECT(smcdet_mh_sweep(&m, &p, &mh, d, d, 1, 4, 10, nullptr, d, d, d, nullptr, d, d, nullptr,
                         nullptr, 0, 0, nullptr, 0, nullptr, nullptr, ws, nullptr, nullptr,
                         nullptr), SMCDET_EINVAL);
  EXPECT(smcdet_mh_sweep(&m, &p, &mh, d, d, 1, 4, 65, nullptr, d, d, d, nullptr, d, d, nullptr,
                         nullptr, 0, 0, nullptr, 0, nullptr, d, ws, nullptr, nullptr, nullptr),
         SMCDET_EUNSUPPORTED);
  // the accept counter is one uint64 per tile: a misaligned workspace is refused
  EXPECT(smcdet_mh_sweep(&m, &p, &mh, d, d, 1, 4, 10, nullptr, d, d, d, nullptr, d, d, nullptr,
                         nullptr, 0, 0, nullptr, 0, nullptr, d, ws + 1, nullptr, nullptr, nullptr),
         SMCDET_EINVAL);
  int64_t anc[4] = {0, 0, 0, 0};
  EXPECT(smcdet_mh_sweep(&m, &p, &mh, d, d, 1, 4, 10, anc, d, d, d, nullptr, d, d, nullptr,
                         nullptr, 0, 0, nullptr, 0, nullptr, d, ws, nullptr, nullptr, nullptr),
         SMCDET_EINVAL);
  smcdet_mh_t bad = mh;
  bad.num_iters = -1;
  EXPECT(smcdet_mh_sweep(&m, &p, &bad, d, d, 1, 4, 10, nullptr, d, d, d, nullptr, dummy + 8,
                         dummy + 12, nullptr, nullptr, 0, 0, nullptr, 0, nullptr, d, ws, nullptr,
                         nullptr, nullptr), SMCDET_EINVAL);
  bad = mh;
  bad.locs_stdev = 0.f;
  EXPECT(smcdet_mh_sweep(&m, &p, &bad, d, d, 1, 4, 10, nullptr, d, d, d, nullptr, dummy + 8,
                         dummy + 12, nullptr, nullptr, 0, 0, nullptr, 0, nullptr, d, ws, nullptr,
                         nullptr, nullptr), SMCDET_EINVAL);
  smcdet_mh_replay_t rp{};
  rp.comp = nullptr;
  EXPECT(smcdet_mh_sweep(&m, &p, &mh, d, d, 1, 4, 10, nullptr, d, d, d, nullptr, dummy + 8,
                         dummy + 12, nullptr, nullptr, 0, 0, &rp, 0, nullptr, d, ws, nullptr,
                         nullptr, nullptr), SMCDET_EINVAL);
  smcdet_image_model_t g = m;
  g.H = g.W = 128;
  EXPECT(smcdet_mh_sweep(&g, &p, &mh, d, d, 1, 4, 10, nullptr, d, d, d, nullptr, dummy + 8,
                         dummy + 12, nullptr, nullptr, 0, 0, nullptr, 0, nullptr, d, ws, nullptr,
                         nullptr, nullptr), SMCDET_EINVAL);
  EXPECT(smcdet_mh_sweep_step(&m, &p, &mh, d, d, 1, 4, 10, nullptr, d, d, d, nullptr, dummy + 8,
                              dummy + 12, nullptr, nullptr, 0, 0, nullptr, 0, d, d, ws, nullptr,
                              nullptr, nullptr, nullptr), SMCDET_EINVAL);
  EXPECT(smcdet_mala_sweep(&g, &p, &mh, d, d, 1, 4, 10, nullptr, d, d, d, nullptr, d, d, nullptr,
                           nullptr, 0, 0, nullptr, 0, nullptr, d, ws, nullptr, nullptr),
         SMCDET_EUNSUPPORTED);
  EXPECT(smcdet_temper(nullptr, d, d, 1, 4, 2.0, nullptr), SMCDET_EINVAL);
  EXPECT(smcdet_temper(d, d, d, 1, 0, 2.0, nullptr), SMCDET_EUNSUPPORTED);
  EXPECT(smcdet_temper(d, d, d, 1, 100000, 2.0, nullptr), SMCDET_EUNSUPPORTED);
  EXPECT(smcdet_update_weights(d, d, d, d, d, nullptr, d, 1, 4, nullptr), SMCDET_EINVAL);
  int64_t idx[4];
  EXPECT(smcdet_resample_index(d, 1, 4, 9, 0, 0, nullptr, idx, nullptr), SMCDET_EINVAL);
  EXPECT(smcdet_temper_reweight(d, d, d, d, d, d, d, 1, 4, 2.0, 9, 0, 0, idx, 0, nullptr, 0,
                                nullptr, nullptr, nullptr, nullptr), SMCDET_EINVAL);
  EXPECT(smcdet_gather(idx, 1, 4, 2, d, d, d, d, d, d, nullptr), SMCDET_EINVAL);
  EXPECT(smcdet_prune(nullptr, d, 1, 1, 1, 8.f, 0.25f, idx, d, d, nullptr), SMCDET_EINVAL);
  EXPECT(smcdet_count_posterior(d, d, 0, 1, 100000, 4, 1, 4, SMCDET_RESAMPLE_SYSTEMATIC, 0, 0,
                                nullptr, nullptr, d, d, d, d, idx, d, d, d, nullptr),
         SMCDET_EUNSUPPORTED);
  EXPECT(smcdet_mh_chain(&m, &p, &mh, d, 1, 1, 10, d, d, d, 100, 200, 1, 0, 10, 0, 0, nullptr, d,
                         d, nullptr, nullptr, nullptr), SMCDET_EINVAL);
  // aggregation: odd joint side, workspace query and requirement
  smcdet_image_model_t j = m;
  j.H = 15;
  EXPECT(smcdet_aggregate_sweep(&j, &p, &mh, 0, d, d, 1, 4, 10, nullptr, d, d, d, nullptr, d, d,
                                0, 0, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr,
                                nullptr, nullptr), SMCDET_EUNSUPPORTED);
  j.H = 128;
  j.W = 64;
  const int64_t need = smcdet_aggregate_workspace(&j, 1, 4, 24);
  if (need != 4 * (2 * 128 * 64 + 3 * 24)) {
    std::printf("FAIL workspace %lld\n", (long long)need);
    ++fails;
  }
  if (smcdet_aggregate_workspace(&m, 1, 4, 10) != 0) ++fails;
  EXPECT(smcdet_aggregate_workspace(&m, 1, 4, 5000), SMCDET_EUNSUPPORTED);
  EXPECT(smcdet_aggregate_sweep(&j, &p, &mh, 0, d, d, 1, 4, 24, nullptr, d, d, d, nullptr, d, d,
                                0, 0, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr,
                                nullptr, nullptr), SMCDET_EINVAL);
  EXPECT(smcdet_aggregate_temper(nullptr, d, d, 1, 1, 4, nullptr, nullptr, nullptr, 0.5, d,
                                 nullptr), SMCDET_EINVAL);
  // timing pool: refuse negative, 0 disables, empty reads
  EXPECT(smcdet_launch_timing(-1), SMCDET_EINVAL);
  EXPECT(smcdet_launch_timing(0), SMCDET_OK);
  float ms[2];
  int32_t n = -1;
  EXPECT(smcdet_launch_timing_read(ms, 2, &n), SMCDET_OK);
  EXPECT(smcdet_launch_timing_starts(ms, 2, &n), SMCDET_OK);
  if (n != 0) ++fails;
  EXPECT(smcdet_host_free(nullptr), SMCDET_OK);  // like free(NULL)
  std::printf("capi sanitizer driver: %d failure(s)\n", fails);
  return fails ? 1 : 0;
}
