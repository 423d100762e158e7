// In-library multi-device context (threading row): ONE process drives several
// GPUs.  The ceremony is sharded by dealer exactly as the one-process-per-GPU path (DESIGN.md section
// 8; dkg_amd/distributed.py): shard i owns dealers dkg_shard_range(n, ndev, i) and runs their share
// generation and round-2/4 checks on its own device (dkg_ceremony_shard_device), one host thread per
// shard.  The exchange step -- every party learns every decision row and the round-3/5 broadcasts
// (committee.rs:311-331, 370-398, 454-467, 790-795) -- needs the rows on ONE device only here,
// because the common outcome is computed once for the process: it is a gather of each shard's
// blocks into device 0's [ws][R][.] arrays by peer copies (xGMI is a full mesh: each copy rides its
// own link, where a ring all-gather would take ws - 1 dependent steps).  Then the combine, the
// round-4 reconstruction on the owning devices (threads again) and the finalise on device 0, with
// the library's own shard entry points, so every output equals the single-GPU and the
// multi-process runs' (tests/test_gpu_multi.py).
//
// A device may appear more than once in `devices`: its shards then share the GPU (the rehearsal of
// the N-device path on a one-GPU box; the peer copies become device-local copies).
#include <hip/hip_runtime_api.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstring>
#include <exception>
#include <map>
#include <string>
#include <thread>
#include <vector>

#include "../../include/dkg_amd.h"

namespace {

struct HipFail {
  std::string what;
};

void hck(hipError_t e, const char* expr) {
  if (e != hipSuccess) throw HipFail{std::string(expr) + ": " + hipGetErrorString(e)};
}
#define MCK(x) hck((x), #x)

struct DevBuf {  // grow-only device allocation
  int dev = 0;
  void* p = nullptr;
  size_t cap = 0;
  void* get(int device, size_t bytes) {
    bytes = bytes ? bytes : 1;
    if (p && cap >= bytes && dev == device) return p;
    MCK(hipSetDevice(device));
    if (p) {
      (void)hipSetDevice(dev);
      (void)hipFree(p);
      p = nullptr;
      MCK(hipSetDevice(device));
    }
    MCK(hipMalloc(&p, bytes));
    dev = device;
    cap = bytes;
    return p;
  }
  void release() {
    if (p) {
      (void)hipSetDevice(dev);
      (void)hipFree(p);
    }
    p = nullptr;
    cap = 0;
  }
};

double now_ms() {
  return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

}  // namespace

struct dkg_multi {
  std::vector<int> dev;
  std::vector<dkg_ctx*> ctx;
  hipStream_t gather = nullptr;  // device 0: the peer copies of the exchange
  std::string err;
  std::map<std::string, double> ms;
  // per shard (on its device): coefficient / broadcast inputs, decision rows, master-key terms,
  // partial final shares
  std::vector<DevBuf> in_a, in_b, in_s, in_sp, dec2, dec4, A0, part;
  // device 0: gathered blocks, compacted matrices, final / public shares
  DevBuf g_dec2, g_dec4, g_A0, g_part, c_dec2, c_dec4, fs, pub;

  int ws() const { return (int)ctx.size(); }
};

namespace {

// Runs f(i) for every shard on its own host thread; the first failing shard's code and message win.
template <class F>
int for_shards(dkg_multi* m, F&& f) {
  const int ws = m->ws();
  std::vector<int> rc(ws, DKG_OK);
  std::vector<std::string> msg(ws);
  std::vector<std::thread> th;
  th.reserve(ws);
  for (int i = 0; i < ws; i++)
    th.emplace_back([&, i] {
      try {
        MCK(hipSetDevice(m->dev[i]));
        rc[i] = f(i);
        if (rc[i] != DKG_OK) msg[i] = dkg_ctx_last_error(m->ctx[i]);
      } catch (const HipFail& x) {
        rc[i] = DKG_E_DEVICE;
        msg[i] = x.what;
      } catch (const std::bad_alloc&) {
        rc[i] = DKG_E_NOMEM;
        msg[i] = "host allocation failed";
      } catch (const std::exception& x) {
        rc[i] = DKG_E_DEVICE;
        msg[i] = x.what();
      }
    });
  for (auto& x : th) x.join();
  for (int i = 0; i < ws; i++)
    if (rc[i] != DKG_OK) {
      m->err = "shard " + std::to_string(i) + " (device " + std::to_string(m->dev[i]) + "): " + msg[i];
      return rc[i];
    }
  return DKG_OK;
}

template <class F>
int guarded_multi(dkg_multi* m, F&& f) {
  if (!m) return DKG_E_ARG;
  try {
    return f();
  } catch (const HipFail& x) {
    m->err = x.what;
    return DKG_E_DEVICE;
  } catch (const std::bad_alloc&) {
    m->err = "host allocation failed";
    return DKG_E_NOMEM;
  }
}

void range(const dkg_multi* m, size_t n, int i, size_t* d0, size_t* d1) { dkg_shard_range(n, m->ws(), i, d0, d1); }

// Gathers every shard's block (bytes_per_row x its dealer count, or `fixed` bytes) into device 0's
// array at block stride `stride`, on the gather stream; returns after the copies completed.
void gather_blocks(dkg_multi* m, size_t n, std::vector<DevBuf>& src, DevBuf& dst, size_t row_bytes, size_t fixed,
                   size_t stride) {
  const int d0dev = m->dev[0];
  MCK(hipSetDevice(d0dev));
  for (int i = 0; i < m->ws(); i++) {
    size_t a, b;
    range(m, n, i, &a, &b);
    const size_t bytes = fixed ? fixed : row_bytes * (b - a);
    if (!bytes) continue;
    uint8_t* to = (uint8_t*)dst.p + stride * i;
    if (m->dev[i] == d0dev)
      MCK(hipMemcpyAsync(to, src[i].p, bytes, hipMemcpyDeviceToDevice, m->gather));
    else
      MCK(hipMemcpyPeerAsync(to, d0dev, src[i].p, m->dev[i], bytes, m->gather));
  }
  MCK(hipStreamSynchronize(m->gather));
}

// The steps after the shards (exchange, combine, reconstruction, finalise) and the host outputs.
int finish(dkg_multi* m, size_t n, size_t t, dkg_ceremony_out* out, double t_start) {
  const int ws = m->ws();
  const int D0 = m->dev[0];
  const size_t R = dkg_shard_rows(n, ws);
  double c0 = now_ms();
  m->g_dec2.get(D0, (size_t)ws * R * n);
  m->g_dec4.get(D0, (size_t)ws * R * n);
  m->g_A0.get(D0, (size_t)ws * R * 32);
  m->g_part.get(D0, (size_t)ws * n * 32);
  gather_blocks(m, n, m->dec2, m->g_dec2, n, 0, R * n);
  gather_blocks(m, n, m->dec4, m->g_dec4, n, 0, R * n);
  gather_blocks(m, n, m->A0, m->g_A0, 32, 0, R * 32);
  gather_blocks(m, n, m->part, m->g_part, 0, 32 * n, 32 * n);
  double c1 = now_ms();
  m->ms["exchange"] = c1 - c0;

  std::vector<uint8_t> q(n), r2e(n), recon(n), r4e(n);
  std::vector<int32_t> c2(n);
  dkg_shard_outcome o{q.data(), c2.data(), r2e.data(), recon.data(), r4e.data(), 0, 0};
  void* cd2 = m->c_dec2.get(D0, n * n);
  void* cd4 = m->c_dec4.get(D0, n * n);
  int rc = dkg_shard_combine_device(m->ctx[0], n, t, ws, m->g_dec2.p, m->g_dec4.p, cd2, cd4, &o);
  if (rc != DKG_OK) {
    m->err = std::string("combine: ") + dkg_ctx_last_error(m->ctx[0]);
    return rc;
  }
  double c2t = now_ms();
  m->ms["combine"] = c2t - c1;

  int no_mpk = o.phase4_error;
  bool any = false;
  for (size_t i = 0; i < n; i++) any |= recon[i] != 0;
  if (any && !o.phase4_error) {
    // a dealer accused in round 4 enters mpk as g * a_i0 over the disclosing final parties'
    // shares (committee.rs:747-789), recovered on the device that holds its share row
    std::vector<int32_t> fail(ws, 0);
    rc = for_shards(m, [&](int i) {
      size_t a, b;
      range(m, n, i, &a, &b);
      return dkg_ceremony_shard_recon_device(m->ctx[i], n, t, a, b, q.data(), recon.data(), r2e.data(), r4e.data(),
                                             nullptr, m->A0[i].p, &fail[i]);
    });
    if (rc != DKG_OK) return rc;
    // every shard derives the verdict from the same gathered outcome: they must agree
    for (int i = 1; i < ws; i++)
      if (fail[i] != fail[0]) {
        m->err = "recon: shards disagree on the recovery outcome";
        return DKG_E_DEVICE;
      }
    no_mpk = fail[0];
    if (!no_mpk) gather_blocks(m, n, m->A0, m->g_A0, 32, 0, R * 32);
  }
  double c3 = now_ms();
  m->ms["recon"] = c3 - c2t;

  void* fs = m->fs.get(D0, 32 * n);
  void* pub = m->pub.get(D0, 32 * n);
  rc = dkg_shard_finalise_device(m->ctx[0], n, t, ws, m->g_A0.p, m->g_part.p, q.data(), no_mpk, fs, pub, out->mpk);
  if (rc != DKG_OK) {
    m->err = std::string("finalise: ") + dkg_ctx_last_error(m->ctx[0]);
    return rc;
  }
  MCK(hipSetDevice(D0));
  if (out->dec2) MCK(hipMemcpy(out->dec2, cd2, n * n, hipMemcpyDeviceToHost));
  if (out->dec4) MCK(hipMemcpy(out->dec4, cd4, n * n, hipMemcpyDeviceToHost));
  if (out->final_share) MCK(hipMemcpy(out->final_share, fs, 32 * n, hipMemcpyDeviceToHost));
  if (out->public_share) MCK(hipMemcpy(out->public_share, pub, 32 * n, hipMemcpyDeviceToHost));
  if (out->qualified) memcpy(out->qualified, q.data(), n);
  if (out->r2_error) memcpy(out->r2_error, r2e.data(), n);
  if (out->r4_error) memcpy(out->r4_error, r4e.data(), n);
  if (out->reconstruct) memcpy(out->reconstruct, recon.data(), n);
  if (out->complaints2) memcpy(out->complaints2, c2.data(), 4 * n);
  out->n_qualified = o.n_qualified;
  out->phase4_error = o.phase4_error;
  if (no_mpk) memset(out->mpk, 0, 32);
  const double end = now_ms();
  m->ms["finalise"] = end - c3;
  out->ms_round1 = 0;
  out->ms_round2 = m->ms["shard_max"];
  out->ms_round3 = c1 - c0;
  out->ms_round4 = c3 - c1;
  out->ms_finalise = end - c3;
  out->ms_total = end - t_start;
  return DKG_OK;
}

int check_args(dkg_multi* m, size_t n, size_t t, dkg_ceremony_out* out) {
  if (!out || dkg_env_check(t, n) != DKG_OK || (size_t)m->ws() > n) {
    m->err = "bad arguments: threshold must be < (n + 1) / 2 (committee.rs:73), out non-NULL, devices <= n";
    return DKG_E_ARG;
  }
  if (out->E || out->A || out->s || out->s_prime) {
    m->err = "E / A / s / s_prime stay on the shards' devices: pass NULL (dkg_ceremony_run returns them)";
    return DKG_E_ARG;
  }
  return DKG_OK;
}

void record_shards(dkg_multi* m, const std::vector<double>& sh) {
  double lo = 1e300, hi = 0;
  for (double x : sh) {
    lo = std::min(lo, x);
    hi = std::max(hi, x);
  }
  m->ms["shard_max"] = hi;
  m->ms["shard_min"] = lo;
}

// shard i's output buffers (on its device)
void shard_outputs(dkg_multi* m, size_t n, int i, size_t D) {
  m->dec2[i].get(m->dev[i], D * n);
  m->dec4[i].get(m->dev[i], D * n);
  m->A0[i].get(m->dev[i], D * 32);
  m->part[i].get(m->dev[i], 32 * n);
}

}  // namespace

extern "C" {

int dkg_multi_create(const int* devices, int ndev, dkg_multi** out) {
  if (!out) return DKG_E_ARG;
  *out = nullptr;
  if (!devices || ndev < 1 || ndev > 64) return DKG_E_ARG;
  int count = dkg_device_count();
  for (int i = 0; i < ndev; i++)
    if (devices[i] < 0 || devices[i] >= count) {
      fprintf(stderr, "dkg_multi_create: device %d is not visible (%d devices)\n", devices[i], count);
      return count ? DKG_E_ARG : DKG_E_DEVICE;
    }
  dkg_multi* m = new dkg_multi();
  m->dev.assign(devices, devices + ndev);
  m->ctx.assign(ndev, nullptr);
  for (auto* v : {&m->in_a, &m->in_b, &m->in_s, &m->in_sp, &m->dec2, &m->dec4, &m->A0, &m->part}) v->resize(ndev);
  int rc = guarded_multi(m, [&] {
    for (int i = 0; i < ndev; i++) {
      int r = dkg_ctx_create(m->dev[i], &m->ctx[i]);
      if (r != DKG_OK) {
        m->err = "dkg_ctx_create(device " + std::to_string(m->dev[i]) + ") failed";
        return r;
      }
    }
    // device 0 pulls every other device's blocks: peer access over xGMI where the pair has it
    // (hipMemcpyPeerAsync stages through the host otherwise)
    MCK(hipSetDevice(m->dev[0]));
    for (int i = 1; i < ndev; i++) {
      if (m->dev[i] == m->dev[0]) continue;
      int can = 0;
      MCK(hipDeviceCanAccessPeer(&can, m->dev[0], m->dev[i]));
      if (can) {
        hipError_t e = hipDeviceEnablePeerAccess(m->dev[i], 0);
        if (e == hipErrorPeerAccessAlreadyEnabled) (void)hipGetLastError();
        else MCK(e);
      }
    }
    MCK(hipStreamCreateWithFlags(&m->gather, hipStreamNonBlocking));
    return DKG_OK;
  });
  if (rc != DKG_OK) {
    fprintf(stderr, "dkg_multi_create: %s\n", m->err.c_str());
    dkg_multi_destroy(m);
    return rc;
  }
  *out = m;
  return DKG_OK;
}

void dkg_multi_destroy(dkg_multi* m) {
  if (!m) return;
  for (auto* v : {&m->in_a, &m->in_b, &m->in_s, &m->in_sp, &m->dec2, &m->dec4, &m->A0, &m->part})
    for (auto& b : *v) b.release();
  for (auto* b : {&m->g_dec2, &m->g_dec4, &m->g_A0, &m->g_part, &m->c_dec2, &m->c_dec4, &m->fs, &m->pub}) b->release();
  if (m->gather) {
    (void)hipSetDevice(m->dev[0]);
    (void)hipStreamDestroy(m->gather);
  }
  for (auto* c : m->ctx) dkg_ctx_destroy(c);
  delete m;
}

int dkg_multi_size(const dkg_multi* m) { return m ? m->ws() : 0; }

dkg_ctx* dkg_multi_ctx(dkg_multi* m, int shard) {
  return m && shard >= 0 && shard < m->ws() ? m->ctx[shard] : nullptr;
}

const char* dkg_multi_last_error(const dkg_multi* m) { return m ? m->err.c_str() : "null multi-device context"; }

double dkg_multi_phase_ms(const dkg_multi* m, const char* name) {
  if (!m || !name) return -1.0;
  auto it = m->ms.find(name);
  return it == m->ms.end() ? -1.0 : it->second;
}

int dkg_multi_env_init(dkg_multi* m, size_t threshold, size_t nr_members, const uint8_t* ck, size_t ck_len,
                       uint8_t h_out[32]) {
  return guarded_multi(m, [&] {
    std::vector<std::vector<uint8_t>> h(m->ws(), std::vector<uint8_t>(32));
    int rc = for_shards(m, [&](int i) {
      return dkg_env_init(m->ctx[i], threshold, nr_members, ck, ck_len, h[i].data());
    });
    if (rc != DKG_OK) return rc;
    if (h_out) memcpy(h_out, h[0].data(), 32);
    return DKG_OK;
  });
}

int dkg_multi_ceremony_run_device(dkg_multi* m, size_t n, size_t t, const void* const* d_a, const void* const* d_b,
                                  dkg_ceremony_out* out) {
  return guarded_multi(m, [&] {
    int rc = check_args(m, n, t, out);
    if (rc != DKG_OK) return rc;
    if (!d_a || !d_b) return DKG_E_ARG;
    const double t0 = now_ms();
    std::vector<double> sh(m->ws(), 0);
    rc = for_shards(m, [&](int i) {
      size_t a, b;
      range(m, n, i, &a, &b);
      shard_outputs(m, n, i, b - a);
      return dkg_ceremony_shard_device(m->ctx[i], n, t, a, b, d_a[i], d_b[i], m->dec2[i].p, m->dec4[i].p,
                                       m->A0[i].p, m->part[i].p, &sh[i]);
    });
    if (rc != DKG_OK) return rc;
    record_shards(m, sh);
    return finish(m, n, t, out, t0);
  });
}

int dkg_multi_ceremony_run(dkg_multi* m, size_t n, size_t t, const uint8_t* a, const uint8_t* b,
                           dkg_ceremony_out* out) {
  return guarded_multi(m, [&] {
    int rc = check_args(m, n, t, out);
    if (rc != DKG_OK) return rc;
    if (!a || !b) return DKG_E_ARG;
    const size_t N = t + 1;
    std::vector<const void*> pa(m->ws()), pb(m->ws());
    rc = for_shards(m, [&](int i) {
      size_t d0, d1;
      range(m, n, i, &d0, &d1);
      const size_t bytes = 32 * N * (d1 - d0);
      pa[i] = m->in_a[i].get(m->dev[i], bytes);
      pb[i] = m->in_b[i].get(m->dev[i], bytes);
      MCK(hipMemcpy((void*)pa[i], a + 32 * N * d0, bytes, hipMemcpyHostToDevice));
      MCK(hipMemcpy((void*)pb[i], b + 32 * N * d0, bytes, hipMemcpyHostToDevice));
      return DKG_OK;
    });
    if (rc != DKG_OK) return rc;
    return dkg_multi_ceremony_run_device(m, n, t, pa.data(), pb.data(), out);
  });
}

int dkg_multi_ceremony_verify(dkg_multi* m, size_t n, size_t t, const uint8_t* E, const uint8_t* A, const uint8_t* s,
                              const uint8_t* s_prime, dkg_ceremony_out* out) {
  return guarded_multi(m, [&] {
    int rc = check_args(m, n, t, out);
    if (rc != DKG_OK) return rc;
    if (!E || !A || !s || !s_prime) return DKG_E_ARG;
    const size_t N = t + 1;
    double t0 = 0;
    std::vector<double> sh(m->ws(), 0);
    // uploads first (every shard), then the timed region
    rc = for_shards(m, [&](int i) {
      size_t d0, d1;
      range(m, n, i, &d0, &d1);
      const size_t D = d1 - d0;
      MCK(hipMemcpy(m->in_a[i].get(m->dev[i], 32 * N * D), E + 32 * N * d0, 32 * N * D, hipMemcpyHostToDevice));
      MCK(hipMemcpy(m->in_b[i].get(m->dev[i], 32 * N * D), A + 32 * N * d0, 32 * N * D, hipMemcpyHostToDevice));
      MCK(hipMemcpy(m->in_s[i].get(m->dev[i], 32 * n * D), s + 32 * n * d0, 32 * n * D, hipMemcpyHostToDevice));
      MCK(hipMemcpy(m->in_sp[i].get(m->dev[i], 32 * n * D), s_prime + 32 * n * d0, 32 * n * D,
                    hipMemcpyHostToDevice));
      shard_outputs(m, n, i, D);
      return DKG_OK;
    });
    if (rc != DKG_OK) return rc;
    t0 = now_ms();
    rc = for_shards(m, [&](int i) {
      size_t d0, d1;
      range(m, n, i, &d0, &d1);
      return dkg_ceremony_shard_verify_device(m->ctx[i], n, t, d0, d1, m->in_a[i].p, m->in_b[i].p, m->in_s[i].p,
                                              m->in_sp[i].p, m->dec2[i].p, m->dec4[i].p, m->A0[i].p, m->part[i].p,
                                              &sh[i]);
    });
    if (rc != DKG_OK) return rc;
    record_shards(m, sh);
    return finish(m, n, t, out, t0);
  });
}

}  // extern "C"
