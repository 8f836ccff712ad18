// Calvin grant groups by key buckets (calvin_bucket.hip): the large-epoch
// path of calvin.hip's request sort + group scan + windowed write-out.
//
// The requests, in sequence order, are partitioned once (stably) into 2^bb
// buckets of the low packed-key bits; each bucket is then finished by one
// workgroup in LDS-sized chunks, in sequence order: a stable LDS radix sort
// of the chunk by the remaining key bits, the grant-group scan with each
// row's state carried from chunk to chunk in an LDS table indexed by those
// bits, and the (request, group) pairs written out partitioned by the txn's
// window of the group array; a last pass places each window in LDS and stores
// it whole, with the txns' readiness.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "radix_sort.h"

namespace dcc {

struct CbPlan {
  uint32_t bb;     // bucket bits (low packed-key bits)
  uint32_t lbits;  // row bits inside a bucket (the LDS carry table has 2^lbits words)
  uint32_t tsh;    // txns per output window = 2^tsh
  uint32_t ndig;   // output windows
  uint32_t ntile;  // partition tiles
  uint32_t R;      // reservation-counter replicas (each with its own pair region)
  uint32_t wt;     // txns per partition wave (1024 / the longest txn)
  uint64_t span;   // requests per window at most (2^tsh * the longest txn)
  uint32_t hashed; // lbits > 13: the carry table is hashed on the row bits (tagged words)
  // workspace sizes in bytes
  uint64_t elem_bytes, out_bytes, cnt_bytes, small_bytes;
};

// The plan for an epoch of n txns x ulen requests (ulen 0: ragged txns of at
// most maxlen requests) with kbits packed key bits; false when the path does
// not apply (wide keys, too many windows).
bool cb_plan(uint64_t n, uint64_t nnz, uint32_t ulen, uint32_t maxlen, uint32_t kbits, CbPlan* p);

struct CbArgs {
  const uint64_t* keys;
  const uint8_t* acctype;
  const uint32_t* seq;  // sequence position -> txn, or null (index order)
  const uint32_t* off;  // index-order offsets (read for ragged txns)
  uint64_t n, nnz;
  uint32_t ulen;        // requests per txn, or 0: ragged
  KeyPack kp;
  // workspaces (CbPlan sizes)
  uint64_t* elems;
  uint64_t* out;
  uint32_t* cnt;
  uint32_t* small;  // tot [2^bb] | bucket base [2^bb] | reservations [R * ndig]
  // outputs
  uint32_t* group;
  uint8_t* rc;
  uint32_t* err;  // CB_ERR_TAB: a hashed carry table ran out of room (redo on the sort path)
};
constexpr uint32_t CB_ERR_TAB = 1u << 12;

// Enqueues the path on st.  ev[0..1] (optional) are recorded after the
// partition and after the bucket pass.
hipError_t cb_run(const CbPlan& p, const CbArgs& a, hipStream_t st, hipEvent_t ev_part,
                  hipEvent_t ev_bucket);

}  // namespace dcc
