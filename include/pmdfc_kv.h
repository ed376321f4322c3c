/*
 * pmdfc_kv.h -- C-ABI of the per-op front-end (libpmdfc_gpucceh.so).
 *
 * The reference's KV front-end is called per op, concurrently, by up to 32
 * RDMA poll threads (server/rdma_svr.cpp:755-835 -> KV::Insert / KV::Get,
 * server/KV.cpp:100-158; NUMA_KV::Insert / Get, server/NuMA_KV.cpp:85-134).
 * These entry points expose the same served path the C++ facades
 * (pmdfc_amd/host/gpu_cceh.h, gpu_cceh_hybrid.h) forward to -- BatchCore: a
 * ring in coherent host memory, a persistent device wave applying the
 * published prefix in ring order, callers reading their own answers -- for
 * non-C++ callers (a ctypes / cgo / JNI binding) and for the op-by-op parity
 * tests.  Plain pointers and sizes; host memory throughout.
 *
 * Order.  The front-end keeps serve_waves rings (one serving wave each); an
 * op goes to the ring of its key's hash prefix, so one key -- and one
 * segment -- always meets the same ring, and ops of different rings touch
 * disjoint segments and commute.  Within ONE ring the ring place is the
 * serial order: the device applies that ring's ops exactly as serial
 * CCEH_hybrid would, in place order.  A place is reported as
 * `place | ring << 48` (places_out).  Ops of one call keep call order only
 * within a ring: a run is split by ring, each piece contiguous in its ring.
 * To replay a stream serially, sort its ops by (ring, place) -- any
 * interleaving of the rings gives the same results and the same table.
 * With serve_waves == 1 there is one ring and call order is the serial order.
 */
#ifndef PMDFC_KV_H_
#define PMDFC_KV_H_

#include <stddef.h>
#include <stdint.h>

#include "pmdfc_cceh.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct pmdfc_kv pmdfc_kv_t;

typedef struct pmdfc_kv_config {
  uint32_t initial_depth;  /* pmdfc_depth_for_hybrid / _src of the reference's initCap */
  uint32_t max_batch;      /* the engine's largest batch (flood batches use it) */
  uint64_t max_segments;   /* 0 = auto */
  int32_t device;
  uint32_t flags;          /* PMDFC_CFG_UPSERT */
  uint32_t ring_size;      /* ring places (rounded up to a power of two, >= 256) */
  uint32_t flood_ops;      /* unanswered places that switch to engine batches (0: never) */
  uint32_t caller_spin_us; /* a blocked caller spins this long, then sleeps */
  uint32_t serve_waves;    /* serving waves (0 = 1); see pmdfc_kv_phase */
} pmdfc_kv_config_t;

int pmdfc_kv_create(const pmdfc_kv_config_t* cfg, pmdfc_kv_t** out);
/* why the calling thread's last pmdfc_kv_create failed ("" if it did not) */
const char* pmdfc_kv_create_error(void);
/* every queued op completes first */
int pmdfc_kv_destroy(pmdfc_kv_t* kv);

/* KV::Insert (server/KV.cpp:100-123) / KV::Get (:145-158) of one op, blocking */
int pmdfc_kv_insert(pmdfc_kv_t* kv, uint64_t key, uint64_t value, uint8_t* status);
int pmdfc_kv_get(pmdfc_kv_t* kv, uint64_t key, uint64_t* value, uint8_t* status);

/* n ops (ops[i]: PMDFC_OP_INSERT / PMDFC_OP_GET) from this thread.
 *   run == 0: one blocking per-op call each (the reference's caller model);
 *   run == k: runs of k ops, each contiguous in the serial order, one wait
 *   per run (BatchCore::MixedRun).
 * values_out: Get values (0 for inserts and misses); places_out (nullable):
 * each op's `place | ring << 48` (see Order above).  Returns the number of failed ops (>= 0) or < 0 on
 * an argument error. */
int64_t pmdfc_kv_ops(pmdfc_kv_t* kv, const uint8_t* ops, const uint64_t* keys, const uint64_t* values_in,
                     uint64_t* values_out, uint8_t* status, uint64_t n, uint32_t run, uint64_t* places_out);
/* The same n ops queued as asynchronous calls (InsertAsync / GetAsync, one
 * callback each writing the op's result), then a wait for all of them.  With
 * many ops in flight the front-end serves the backlog as engine batches (the
 * flood hand-off, pmdfc_kv_config_t.flood_ops). */
int64_t pmdfc_kv_ops_async(pmdfc_kv_t* kv, const uint8_t* ops, const uint64_t* keys, const uint64_t* values_in,
                           uint64_t* values_out, uint8_t* status, uint64_t n, uint64_t* places_out);
/* wait for every op queued before the call */
int pmdfc_kv_flush(pmdfc_kv_t* kv);

/* CCEH::Utilization / Capacity / FindAnyway after every queued op
 * (CCEH_hybrid.cpp:412-435, 482-496) */
int pmdfc_kv_utilization(pmdfc_kv_t* kv, double* out);
int pmdfc_kv_capacity(pmdfc_kv_t* kv, uint64_t* out);
int pmdfc_kv_find_anyway(pmdfc_kv_t* kv, uint64_t key, uint64_t* value, uint8_t* status);
/* the index after every queued op (the serving waves stopped meanwhile):
 * pmdfc_cceh_stats, and pmdfc_cceh_dump's canonical dump sized and filled
 * under ONE stop of the waves (ABI 8: other threads' ops may split segments
 * between two calls, so the dump checks the buffers itself).  dir_cap:
 * entries of dir_canon; seg_cap: entries of local_depth / prefix, and
 * seg_cap * 1024 of keys / values.  *nseg_out / *ndir_out (nullable)
 * receive the sizes; buffers too small -> PMDFC_ERR_SIZE, nothing written
 * (call again with larger ones).  Any buffer may be NULL (sizes only). */
int pmdfc_kv_stats(pmdfc_kv_t* kv, pmdfc_cceh_stats_t* out);
int pmdfc_kv_dump(pmdfc_kv_t* kv, uint64_t dir_cap, uint64_t seg_cap, uint32_t* dir_canon, uint32_t* local_depth,
                  uint64_t* prefix, uint64_t* keys, uint64_t* values, uint64_t* nseg_out, uint64_t* ndir_out);
/* counters: [0] serving-wave launches, [1] device chunks (wave chunks +
 * flood batches), [2] flood batches, [3] ops in flood batches, [4] failed
 * ops, [5] ops completed, [6] serving waves per launch, [7] header reloads
 * of the serving waves (chunks whose ordered path may have changed a
 * directory bucket header) */
#define PMDFC_KV_NPHASE 8
int pmdfc_kv_phase(pmdfc_kv_t* kv, uint64_t* out);
const char* pmdfc_kv_last_error(pmdfc_kv_t* kv);

#ifdef __cplusplus
}
#endif
#endif /* PMDFC_KV_H_ */
