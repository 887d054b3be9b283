// Bench/test tooling (not the engine): the deterministic RMAT generator of nebula_amd/rmat.py
// restated in C++/OpenMP so RMAT-22..26 inputs are produced in seconds.  Bit-identical to the
// numpy version (tests/test_rmat.py checks it).
#include <omp.h>

#include <cstdint>
#include <vector>

namespace {
inline uint64_t mix(uint64_t z) {
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}
inline uint64_t splitmix64(uint64_t x) { return mix(x + 0x9E3779B97F4A7C15ull); }
}  // namespace

extern "C" int nbgtool_rmat(int scale, int edge_factor, uint64_t seed, int64_t* src, int64_t* dst, int64_t* w) {
  const uint64_t n = (uint64_t)edge_factor << scale;
  const uint64_t ta = (uint64_t)(0.57 * 9007199254740992.0);
  const uint64_t tab = (uint64_t)((0.57 + 0.19) * 9007199254740992.0);
  const uint64_t tabc = (uint64_t)((0.57 + 0.19 + 0.19) * 9007199254740992.0);
#pragma omp parallel for schedule(static, 65536)
  for (int64_t ii = 0; ii < (int64_t)n; ++ii) {
    uint64_t i = (uint64_t)ii, u = 0, v = 0, base = i * 64;
    for (int l = 0; l < scale; ++l) {
      uint64_t r = splitmix64(seed ^ (base + (uint64_t)l)) >> 11;
      uint64_t bu = r >= tab;
      uint64_t bv = ((r >= ta) && (r < tab)) || (r >= tabc);
      u |= bu << l;
      v |= bv << l;
    }
    src[i] = (int64_t)(mix(u + seed) & 0x7FFFFFFFFFFFFFFFull);
    dst[i] = (int64_t)(mix(v + seed) & 0x7FFFFFFFFFFFFFFFull);
    w[i] = (int64_t)(splitmix64(seed ^ ~i) % 100);
  }
  return 0;
}

// Vertex sets of the same graph without sorting the sample arrays: marks src_seen[u] / any_seen[u]
// over the RMAT id space (u < 2^scale; the vid is mix(u + seed) masked, as above).  Byte stores
// of the same value from several threads are benign.
extern "C" int nbgtool_rmat_vertices(int scale, int edge_factor, uint64_t seed, uint8_t* src_seen, uint8_t* any_seen) {
  const uint64_t n = (uint64_t)edge_factor << scale;
  const uint64_t ta = (uint64_t)(0.57 * 9007199254740992.0);
  const uint64_t tab = (uint64_t)((0.57 + 0.19) * 9007199254740992.0);
  const uint64_t tabc = (uint64_t)((0.57 + 0.19 + 0.19) * 9007199254740992.0);
#pragma omp parallel for schedule(static, 65536)
  for (int64_t ii = 0; ii < (int64_t)n; ++ii) {
    uint64_t i = (uint64_t)ii, u = 0, v = 0, base = i * 64;
    for (int l = 0; l < scale; ++l) {
      uint64_t r = splitmix64(seed ^ (base + (uint64_t)l)) >> 11;
      uint64_t bu = r >= tab;
      uint64_t bv = ((r >= ta) && (r < tab)) || (r >= tabc);
      u |= bu << l;
      v |= bv << l;
    }
    src_seen[u] = 1;
    any_seen[u] = 1;
    any_seen[v] = 1;
  }
  return 0;
}

// vid of RMAT id u (the scramble above), for ids u[0..n)
extern "C" int nbgtool_rmat_vids(uint64_t seed, const uint64_t* u, uint64_t n, int64_t* out) {
#pragma omp parallel for schedule(static)
  for (int64_t i = 0; i < (int64_t)n; ++i) out[i] = (int64_t)(mix(u[i] + seed) & 0x7FFFFFFFFFFFFFFFull);
  return 0;
}

// The samples of the same graph a partitioned rank keeps: those whose source or destination lives
// on GPU `rank` of `gpus` (part = (uint64)vid % parts + 1, GPU = part % gpus; the loader keeps
// out-edges at the source's part and in-edges at the destination's), in sample order, so that
// "the last of duplicate samples wins" is unchanged.  A rank then holds about 2/gpus of the
// samples instead of all of them.  src == nullptr: returns the count only.
extern "C" int64_t nbgtool_rmat_owned(int scale, int edge_factor, uint64_t seed, int parts, int gpus, int rank,
                                      int64_t* src, int64_t* dst, int64_t* w) {
  const uint64_t n = (uint64_t)edge_factor << scale;
  const uint64_t ta = (uint64_t)(0.57 * 9007199254740992.0);
  const uint64_t tab = (uint64_t)((0.57 + 0.19) * 9007199254740992.0);
  const uint64_t tabc = (uint64_t)((0.57 + 0.19 + 0.19) * 9007199254740992.0);
  constexpr uint64_t CH = 65536;
  const uint64_t nch = (n + CH - 1) / CH;
  auto sample = [&](uint64_t i, int64_t* s, int64_t* d) {
    uint64_t u = 0, v = 0, base = i * 64;
    for (int l = 0; l < scale; ++l) {
      uint64_t r = splitmix64(seed ^ (base + (uint64_t)l)) >> 11;
      uint64_t bu = r >= tab;
      uint64_t bv = ((r >= ta) && (r < tab)) || (r >= tabc);
      u |= bu << l;
      v |= bv << l;
    }
    *s = (int64_t)(mix(u + seed) & 0x7FFFFFFFFFFFFFFFull);
    *d = (int64_t)(mix(v + seed) & 0x7FFFFFFFFFFFFFFFull);
  };
  auto owned = [&](int64_t vid) { return (int)(((uint64_t)vid % (uint64_t)parts + 1) % (uint64_t)gpus) == rank; };
  std::vector<int64_t> cnt(nch + 1, 0);
#pragma omp parallel for schedule(static, 1)
  for (int64_t c = 0; c < (int64_t)nch; ++c) {
    int64_t k = 0;
    const uint64_t e = ((uint64_t)c + 1) * CH < n ? ((uint64_t)c + 1) * CH : n;
    for (uint64_t i = (uint64_t)c * CH; i < e; ++i) {
      int64_t s, d;
      sample(i, &s, &d);
      k += owned(s) || owned(d);
    }
    cnt[c + 1] = k;
  }
  for (uint64_t c = 0; c < nch; ++c) cnt[c + 1] += cnt[c];
  if (!src) return cnt[nch];
#pragma omp parallel for schedule(static, 1)
  for (int64_t c = 0; c < (int64_t)nch; ++c) {
    int64_t o = cnt[c];
    const uint64_t e = ((uint64_t)c + 1) * CH < n ? ((uint64_t)c + 1) * CH : n;
    for (uint64_t i = (uint64_t)c * CH; i < e; ++i) {
      int64_t s, d;
      sample(i, &s, &d);
      if (!(owned(s) || owned(d))) continue;
      src[o] = s;
      dst[o] = d;
      w[o] = (int64_t)(splitmix64(seed ^ ~i) % 100);
      ++o;
    }
  }
  return cnt[nch];
}
