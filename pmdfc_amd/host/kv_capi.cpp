// kv_capi.cpp -- the C-ABI of the per-op front-end (include/pmdfc_kv.h) over
// BatchCore (batch_core.h): what KV::Insert / KV::Get (server/KV.cpp:100-158)
// call per op, for callers that bind C rather than the C++ facades.
#include <cstring>
#include <memory>
#include <new>
#include <string>
#include <vector>

#include "../../include/pmdfc_kv.h"
#include "batch_core.h"

struct pmdfc_kv {
  std::unique_ptr<pmdfc_host::BatchCore> core;
  std::string err;
};

namespace {

thread_local std::string create_err;  // pmdfc_kv_create_error

// one async op's result slot
struct Slot {
  uint64_t* vout;
  uint8_t* st;
};

void slot_cb(void* ctx, uint8_t status, uint64_t value) {
  Slot* s = static_cast<Slot*>(ctx);
  *s->st = status;
  if (s->vout) *s->vout = value;
}

}  // namespace

extern "C" {

int pmdfc_kv_create(const pmdfc_kv_config_t* cfg, pmdfc_kv_t** out) {
  if (!cfg || !out) return PMDFC_ERR_ARG;
  *out = nullptr;
  pmdfc_host::BatchingConfig c;
  if (cfg->max_batch) c.max_batch = cfg->max_batch;
  c.device = cfg->device;
  c.upsert = (cfg->flags & PMDFC_CFG_UPSERT) != 0;
  if (cfg->ring_size) c.ring_size = cfg->ring_size;
  c.flood_ops = cfg->flood_ops;
  if (cfg->caller_spin_us) c.caller_spin_us = cfg->caller_spin_us;
  c.serve_waves = cfg->serve_waves ? cfg->serve_waves : 1u;
  create_err.clear();
  pmdfc_kv* kv = new (std::nothrow) pmdfc_kv;
  if (!kv) {
    create_err = "out of host memory";
    return PMDFC_ERR_NOMEM;
  }
  try {
    kv->core.reset(new pmdfc_host::BatchCore(cfg->initial_depth, c, cfg->max_segments));
  } catch (const std::exception& e) {
    create_err = e.what();  // (BatchCore released what it had allocated)
    delete kv;
    return PMDFC_ERR_HIP;
  }
  *out = kv;
  return PMDFC_OK;
}

int pmdfc_kv_destroy(pmdfc_kv_t* kv) {
  delete kv;
  return PMDFC_OK;
}

int pmdfc_kv_insert(pmdfc_kv_t* kv, uint64_t key, uint64_t value, uint8_t* status) {
  if (!kv) return PMDFC_ERR_ARG;
  const uint8_t st = kv->core->Insert(key, value);
  if (status) *status = st;
  return PMDFC_OK;
}

int pmdfc_kv_get(pmdfc_kv_t* kv, uint64_t key, uint64_t* value, uint8_t* status) {
  if (!kv) return PMDFC_ERR_ARG;
  const uint8_t st = kv->core->Get(key, value);
  if (status) *status = st;
  return PMDFC_OK;
}

int64_t pmdfc_kv_ops(pmdfc_kv_t* kv, const uint8_t* ops, const uint64_t* keys, const uint64_t* values_in,
                     uint64_t* values_out, uint8_t* status, uint64_t n, uint32_t run, uint64_t* places_out) {
  if (!kv || (n && (!ops || !keys || !values_in || !status))) return PMDFC_ERR_ARG;
  uint64_t bad = 0;
  const uint64_t step = run ? run : 1;
  for (uint64_t o = 0; o < n; o += step) {
    const uint64_t m = n - o < step ? n - o : step;
    bad += kv->core->MixedRun(ops + o, keys + o, values_in + o, values_out ? values_out + o : nullptr, status + o, m,
                              places_out ? places_out + o : nullptr);
  }
  return (int64_t)bad;
}

int64_t pmdfc_kv_ops_async(pmdfc_kv_t* kv, const uint8_t* ops, const uint64_t* keys, const uint64_t* values_in,
                           uint64_t* values_out, uint8_t* status, uint64_t n, uint64_t* places_out) {
  if (!kv || (n && (!ops || !keys || !values_in || !status))) return PMDFC_ERR_ARG;
  std::vector<Slot> slots(n);
  for (uint64_t i = 0; i < n; ++i) {
    slots[i] = Slot{values_out ? values_out + i : nullptr, status + i};
    status[i] = pmdfc_host::kBatchFailed;
    if (values_out) values_out[i] = 0;
    const uint64_t p = kv->core->SubmitAsync(ops[i], keys[i], values_in[i], slot_cb, &slots[i]);
    if (places_out) places_out[i] = p;
  }
  if (!kv->core->flush()) return PMDFC_ERR_STATE;
  int64_t bad = 0;
  for (uint64_t i = 0; i < n; ++i) bad += pmdfc_host::BatchCore::is_failure(ops[i], status[i]) ? 1 : 0;
  return bad;
}

int pmdfc_kv_flush(pmdfc_kv_t* kv) {
  if (!kv) return PMDFC_ERR_ARG;
  return kv->core->flush() ? PMDFC_OK : PMDFC_ERR_STATE;
}

int pmdfc_kv_utilization(pmdfc_kv_t* kv, double* out) {
  if (!kv || !out) return PMDFC_ERR_ARG;
  *out = kv->core->Utilization();
  return *out < 0 ? PMDFC_ERR_STATE : PMDFC_OK;
}

int pmdfc_kv_capacity(pmdfc_kv_t* kv, uint64_t* out) {
  if (!kv || !out) return PMDFC_ERR_ARG;
  *out = kv->core->Capacity();
  return PMDFC_OK;
}

int pmdfc_kv_find_anyway(pmdfc_kv_t* kv, uint64_t key, uint64_t* value, uint8_t* status) {
  if (!kv) return PMDFC_ERR_ARG;
  uint64_t v = 0;
  const uint8_t st = kv->core->FindAnyway(key, &v);
  if (value) *value = st == PMDFC_ST_HIT ? v : 0;
  if (status) *status = st;
  return st == pmdfc_host::kBatchFailed ? PMDFC_ERR_STATE : PMDFC_OK;
}

int pmdfc_kv_stats(pmdfc_kv_t* kv, pmdfc_cceh_stats_t* out) {
  if (!kv || !out) return PMDFC_ERR_ARG;
  return kv->core->Stats(out);
}

const char* pmdfc_kv_create_error(void) { return create_err.c_str(); }

int pmdfc_kv_dump(pmdfc_kv_t* kv, uint64_t dir_cap, uint64_t seg_cap, uint32_t* dir_canon, uint32_t* local_depth,
                  uint64_t* prefix, uint64_t* keys, uint64_t* values, uint64_t* nseg_out, uint64_t* ndir_out) {
  if (!kv) return PMDFC_ERR_ARG;
  return kv->core->Dump(dir_cap, seg_cap, dir_canon, local_depth, prefix, keys, values, nseg_out, ndir_out);
}

int pmdfc_kv_phase(pmdfc_kv_t* kv, uint64_t* out) {
  if (!kv || !out) return PMDFC_ERR_ARG;
  const auto ph = kv->core->phase_times();
  out[0] = ph.wave_starts;
  out[1] = ph.batches;
  out[2] = ph.flood_batches;
  out[3] = ph.flood_ops;
  out[4] = kv->core->failed_ops();
  out[5] = kv->core->ops_completed();
  out[6] = kv->core->serve_waves();
  out[7] = kv->core->header_reloads();
  return PMDFC_OK;
}

const char* pmdfc_kv_last_error(pmdfc_kv_t* kv) {
  if (!kv) return "null handle";
  kv->err = kv->core->last_error();
  return kv->err.c_str();
}

}  // extern "C"
