// common.hip — error state, version, model pre-digestion for the C ABI.
#include <string.h>
#include <math.h>
#include <stdarg.h>
#include <stdio.h>

#include "device.h"

namespace smcdet {

static thread_local char g_err[512] = "";

int set_error(int code, const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
  return code;
}

int check_launch(const char* what) {
  hipError_t e = hipGetLastError();
  if (e != hipSuccess)
    return set_error(SMCDET_EHIP, "%s: %s", what, hipGetErrorString(e));
  return SMCDET_OK;
}

int ensure_lds(const void* kernel, size_t bytes) {
  if (bytes > 160 * 1024)
    return set_error(SMCDET_EUNSUPPORTED, "kernel needs %zu B of LDS (> 160 KiB)", bytes);
  if (bytes > 64 * 1024 &&
      hipFuncSetAttribute(kernel, hipFuncAttributeMaxDynamicSharedMemorySize, (int)bytes) !=
          hipSuccess)
    return set_error(SMCDET_EHIP, "hipFuncSetAttribute(%zu B LDS) failed", bytes);
  return SMCDET_OK;
}

// ---- launch timing pool (smcdet_launch_timing / _read) ----------------------
static hipEvent_t* g_tev = nullptr;  // 2 * g_tcap events: (start, stop) per launch
static int g_tcap = 0, g_tused = 0;
static bool g_ttiles = false;  // smcdet_launch_timing_tiles

bool timing_tiles() { return g_ttiles && g_tused < g_tcap; }

bool timing_next(hipEvent_t* start, hipEvent_t* stop) {
  if (g_tused >= g_tcap) return false;
  *start = g_tev[2 * g_tused];
  *stop = g_tev[2 * g_tused + 1];
  ++g_tused;
  return true;
}

static void timing_free() {
  for (int i = 0; i < 2 * g_tcap; ++i) (void)hipEventDestroy(g_tev[i]);
  delete[] g_tev;
  g_tev = nullptr;
  g_tcap = g_tused = 0;
  g_ttiles = false;
}

int validate_model(const smcdet_image_model_t* m, int max_pixels) {
  if (!m) return set_error(SMCDET_EINVAL, "image model is null");
  if (m->model != SMCDET_MODEL_M71 && m->model != SMCDET_MODEL_POISSON)
    return set_error(SMCDET_EINVAL, "unknown image model %d", m->model);
  if (m->H <= 0 || m->W <= 0 || (int64_t)m->H * m->W > max_pixels)
    return set_error(SMCDET_EUNSUPPORTED, "tile %dx%d outside 1..%d pixels", m->H, m->W,
                     max_pixels);
  if (m->model == SMCDET_MODEL_POISSON && m->H * m->W > kMaxLdsPixels)
    return set_error(SMCDET_EUNSUPPORTED,
                     "tile %dx%d: tiles above %d pixels run the M71 image model only", m->H,
                     m->W, kMaxLdsPixels);
  if (m->psf_radius < 0 || m->psf_radius > 64)
    return set_error(SMCDET_EUNSUPPORTED, "psf_radius %d outside 0..64", m->psf_radius);
  return SMCDET_OK;
}

DevModel make_dev_model(const smcdet_image_model_t& m) {
  DevModel d{};
  d.model = m.model;
  d.H = m.H;
  d.W = m.W;
  d.R = m.psf_radius;
  d.bg = m.background;
  if (m.model == SMCDET_MODEL_M71) {
    const double s1 = m.psf_params[0], s2 = m.psf_params[1], sp = m.psf_params[2];
    const double beta = m.psf_params[3], b = m.psf_params[4], p0 = m.psf_params[5];
    const double log2e = 1.4426950408889634;
    d.g = m.adu_per_nmgy;
    d.k1 = (float)(-log2e / (2.0 * s1));
    d.k2 = (float)(-log2e / (2.0 * s2));
    d.b = (float)b;
    d.k3 = (float)(1.0 / (beta * sp));
    d.kb = (float)(-beta / 2.0);
    d.p0 = (float)p0;
    d.inv_norm = (float)(1.0 / ((1.0 + b + p0) * (double)m.psf_norm));
    d.lb2 = b > 0 ? (float)log2(b) : -INFINITY;
    d.lp02 = p0 > 0 ? (float)log2(p0) : -INFINITY;
    d.s0sq = m.noise_additive;
    d.eta = m.noise_multiplicative;
  } else {
    const double s = m.psf_params[0];
    d.g = 1.0f;
    d.kg = (float)(-1.4426950408889634 / (2.0 * s * s));
    d.amp = (float)(1.0 / (s * sqrt(2.0 * M_PI)));
  }
  return d;
}

DevPrior make_dev_prior(const smcdet_prior_t& p) {
  DevPrior d{};
  d.kind = p.kind;
  d.lo = p.loc_low;
  d.lo_w = p.loc_low;
  d.hi_h = p.loc_high_h;
  d.hi_w = p.loc_high_w;
  d.min_objects = p.min_objects;
  d.max_objects = p.max_objects;
  d.alpha = p.flux_alpha;
  d.lower = p.flux_lower;
  d.upper = p.flux_upper;
  d.ap1 = (float)((double)p.flux_alpha + 1.0);
  d.loc_lp_h = (float)(-log((double)p.loc_high_h - (double)p.loc_low));
  d.loc_lp_w = (float)(-log((double)p.loc_high_w - (double)p.loc_low));
  const double a = p.flux_alpha, L = p.flux_lower, U = p.flux_upper;
  if (p.kind == SMCDET_PRIOR_M71) {
    d.count_c0 = (float)log((double)p.poisson_mean);
    d.count_c1 = p.poisson_mean;
    // TruncatedPareto.logpdf_norm_const (distributions.py:69-74)
    d.flux_c = (float)(log(a) + a * log(L) + a * log(U) - log(pow(U, a) - pow(L, a)));
  } else {
    d.count_c0 = (float)log(1.0 / (double)(p.max_objects - p.min_objects + 1));
    // Pareto(scale, alpha).log_prob: log(alpha) + alpha*log(scale) - (alpha+1)*log(f)
    d.flux_c = (float)(log(a) + a * log(L));
  }
  return d;
}

int validate_prior(const smcdet_prior_t* p) {
  if (!p) return set_error(SMCDET_EINVAL, "prior is null");
  if (p->kind != SMCDET_PRIOR_M71 && p->kind != SMCDET_PRIOR_PARETO)
    return set_error(SMCDET_EINVAL, "unknown prior kind %d", p->kind);
  if (p->min_objects < 0 || p->max_objects < p->min_objects || p->max_objects > 4096)
    return set_error(SMCDET_EUNSUPPORTED, "objects %d..%d outside 0..4096", p->min_objects,
                     p->max_objects);
  return SMCDET_OK;
}

}  // namespace smcdet

extern "C" {

int smcdet_launch_timing(int32_t max_launches) {
  smcdet::timing_free();
  if (max_launches < 0) return smcdet::set_error(SMCDET_EINVAL, "max_launches < 0");
  if (max_launches == 0) return SMCDET_OK;
  smcdet::g_tev = new hipEvent_t[2 * (size_t)max_launches];
  for (int i = 0; i < 2 * max_launches; ++i) {
    if (hipEventCreate(&smcdet::g_tev[i]) != hipSuccess) {
      for (int k = 0; k < i; ++k) (void)hipEventDestroy(smcdet::g_tev[k]);
      delete[] smcdet::g_tev;
      smcdet::g_tev = nullptr;
      return smcdet::set_error(SMCDET_EHIP, "hipEventCreate failed");
    }
  }
  smcdet::g_tcap = max_launches;
  smcdet::g_tused = 0;
  return SMCDET_OK;
}

int smcdet_launch_timing_read(float* ms, int32_t max, int32_t* n_out) {
  const int n = smcdet::g_tused < max ? smcdet::g_tused : max;
  for (int i = 0; i < n; ++i) {
    if (hipEventSynchronize(smcdet::g_tev[2 * i + 1]) != hipSuccess ||
        hipEventElapsedTime(&ms[i], smcdet::g_tev[2 * i], smcdet::g_tev[2 * i + 1]) != hipSuccess)
      return smcdet::set_error(SMCDET_EHIP, "launch %d: event timing failed", i);
  }
  if (n_out) *n_out = smcdet::g_tused;
  return SMCDET_OK;
}

int smcdet_launch_timing_starts(float* ms, int32_t max, int32_t* n_out) {
  const int n = smcdet::g_tused < max ? smcdet::g_tused : max;
  for (int i = 0; i < n; ++i) {
    if (hipEventSynchronize(smcdet::g_tev[2 * i]) != hipSuccess ||
        hipEventElapsedTime(&ms[i], smcdet::g_tev[0], smcdet::g_tev[2 * i]) != hipSuccess)
      return smcdet::set_error(SMCDET_EHIP, "launch %d: event timing failed", i);
  }
  if (n_out) *n_out = smcdet::g_tused;
  return SMCDET_OK;
}

int smcdet_launch_timing_tiles(int32_t on) {
  smcdet::g_ttiles = on != 0;
  return SMCDET_OK;
}

#ifndef SMCDET_SRC_HASH
#define SMCDET_SRC_HASH "unknown"
#endif
// "src <sha1>": the sha1 of the library's sources (Makefile SRC_HASH)
// the diagnostic build (make diag) says so: "(gfx950, diag)"
#ifdef SMCDET_DIAG
#define SMCDET_BUILD_KIND ", diag"
#else
#define SMCDET_BUILD_KIND ""
#endif
const char* smcdet_version(void) {
  return "smcdet_hip 0.2.0 (gfx950" SMCDET_BUILD_KIND ") src " SMCDET_SRC_HASH;
}
int32_t smcdet_abi_version(void) { return SMCDET_ABI_VERSION; }
const char* smcdet_last_error(void) { return smcdet::g_err; }

int smcdet_host_alloc(size_t bytes, void** host, void** device) {
  using namespace smcdet;
  if (!host || !device || bytes == 0) return set_error(SMCDET_EINVAL, "bad host_alloc args");
  *host = nullptr;
  *device = nullptr;
  if (hipHostMalloc(host, bytes, hipHostMallocMapped) != hipSuccess)
    return set_error(SMCDET_EHIP, "hipHostMalloc(%zu) failed", bytes);
  if (hipHostGetDevicePointer(device, *host, 0) != hipSuccess) {
    (void)hipHostFree(*host);
    *host = nullptr;
    return set_error(SMCDET_EHIP, "hipHostGetDevicePointer failed");
  }
  memset(*host, 0, bytes);
  return SMCDET_OK;
}

int smcdet_host_free(void* host) {
  if (host && hipHostFree(host) != hipSuccess)
    return smcdet::set_error(SMCDET_EHIP, "hipHostFree failed");
  return SMCDET_OK;
}

}  // extern "C"
