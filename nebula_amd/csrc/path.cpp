// FIND SHORTEST | ALL PATH driver (FindPathExecutor semantics).
#include "engine.h"

extern "C" int32_t nbg_find_path(nbg_engine* h, const nbg_path_request* req, nbg_paths** out) {
  if (!h || !req || !out) return NBG_E_INVALID_ARGUMENT;
  *out = nullptr;
  return h->e.fail(NBG_E_UNSUPPORTED, "FIND PATH device path not built yet");
}

extern "C" int32_t nbg_comm_unique_id(uint8_t out[NBG_UNIQUE_ID_BYTES]) {
  (void)out;
  return NBG_E_UNSUPPORTED;
}

extern "C" int32_t nbg_comm_init(nbg_engine* h, const uint8_t id[NBG_UNIQUE_ID_BYTES], int32_t world, int32_t rank) {
  (void)id; (void)world; (void)rank;
  return h ? h->e.fail(NBG_E_UNSUPPORTED, "multi-GPU not built yet") : NBG_E_INVALID_ARGUMENT;
}
