// Host-side key sharding helpers: GPU g owns the keys with
// dcc_key_shard(key, G) == g — the node striping GET_NODE_ID (global.h:294)
// recast as a hash so zipf-hot keys spread over the GPUs.
#include <cstring>

#include "dcc.h"
#include "dcc_internal.h"

extern "C" uint32_t dcc_key_shard(uint64_t key, uint32_t nranks) {
  if (nranks <= 1) return 0;
  // splitmix64 finaliser; independent of the device table hash (fmix64)
  const uint64_t h = dcc::splitmix64(key ^ 0x5DEECE66Dull);
  return (uint32_t)((((unsigned __int128)h) * nranks) >> 64);
}

extern "C" int dcc_key_shard_n(const uint64_t* keys, uint64_t n, uint32_t nranks, uint32_t* out) {
  if ((n && (!keys || !out)) || nranks == 0) return DCC_EINVAL;
  for (uint64_t i = 0; i < n; i++) out[i] = dcc_key_shard(keys[i], nranks);
  return DCC_OK;
}

extern "C" int dcc_shard_filter(const dcc_batch* in, uint32_t rank, uint32_t nranks,
                                uint32_t* out_offsets, uint64_t* out_keys, uint8_t* out_acctype,
                                uint64_t* out_nnz) {
  if (!in || !out_offsets || !out_nnz || nranks == 0 || rank >= nranks) return DCC_EINVAL;
  if (in->flags & (DCC_DEVICE_PTRS | DCC_COMPACT_FLAGS)) return DCC_EINVAL;  // full-width host batches
  if (in->nnz && (!in->keys || !in->acctype || !out_keys || !out_acctype)) return DCC_EINVAL;
  uint64_t w = 0;
  out_offsets[0] = 0;
  for (uint64_t t = 0; t < in->n_txn; t++) {
    for (uint32_t x = in->offsets[t]; x < in->offsets[t + 1]; x++) {
      if (dcc_key_shard(in->keys[x], nranks) != rank) continue;
      out_keys[w] = in->keys[x];
      out_acctype[w] = in->acctype[x];
      w++;
    }
    out_offsets[t + 1] = (uint32_t)w;
  }
  *out_nnz = w;
  return DCC_OK;
}
