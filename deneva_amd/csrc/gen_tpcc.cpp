// TPC-C batch producer — placeholder until the NewOrder/Payment restatement lands.
#include <cstring>

#include "dcc.h"

extern "C" void dcc_tpcc_params_default(dcc_tpcc_params* p) {
  memset(p, 0, sizeof(*p));
  p->n_txn = 262144;
  p->num_wh = 128;
  p->part_cnt = 1;
  p->perc_payment = 0.5;
  p->wh_update = 1;
  p->max_items = 100000;
  p->cust_per_dist = 3000;
  p->dist_per_wh = 10;
  p->max_items_per_txn = 15;
  p->part_per_txn = 1;
  p->mpr = 1.0;
  p->first_part_local = 1;
  p->chunk_txns = 65536;
  p->seed = 0xD3E7A003ull;
}
extern "C" uint32_t dcc_tpcc_max_access(const dcc_tpcc_params* p) {
  return 3 + 2 * (p ? p->max_items_per_txn : 15);
}
extern "C" int dcc_gen_tpcc(const dcc_tpcc_params*, uint32_t*, uint64_t*, uint8_t*, uint8_t*,
                            uint64_t*) {
  return DCC_ENOTSUP;
}
