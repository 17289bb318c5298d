// z-slab decomposition of one volume over the ranks of a Comm (include/nm03/volume_slabs.h).
#include "nm03/volume_slabs.h"

#include <algorithm>
#include <cstring>

#include "nm03/golden.h"

namespace nm03 {

namespace {

size_t plane_words(int w, int h) { return (size_t)h * (size_t)((w + 63) / 64); }

int64_t popcount(const std::vector<uint64_t>& v) {
  int64_t n = 0;
  for (uint64_t x : v) n += __builtin_popcountll(x);
  return n;
}

std::vector<uint8_t> to_bytes(const std::vector<std::vector<uint64_t>>& planes) {
  std::vector<uint8_t> b;
  for (const auto& p : planes) {
    const auto* s = reinterpret_cast<const uint8_t*>(p.data());
    b.insert(b.end(), s, s + p.size() * 8);
  }
  return b;
}

std::vector<std::vector<uint64_t>> from_bytes(const uint8_t* b, size_t nplanes, size_t pw) {
  std::vector<std::vector<uint64_t>> out(nplanes, std::vector<uint64_t>(pw));
  for (size_t k = 0; k < nplanes; ++k) std::memcpy(out[k].data(), b + k * pw * 8, pw * 8);
  return out;
}

}  // namespace

std::vector<Seed> slab_seeds(const std::vector<Seed>& seeds, int w, int h, int depth, int z0, int d) {
  std::vector<Seed> all = seeds;
  if (all.empty()) {
    all = reference_seeds(w, h);
    for (auto& s : all) s.z = depth / 2;
  }
  std::vector<Seed> out;
  for (const Seed& s : all)
    if (s.z >= z0 && s.z < z0 + d) out.push_back(Seed{s.x, s.y, s.z - z0});
  return out;
}

std::vector<uint64_t> pack_plane(const uint8_t* px, int w, int h) {
  const int n = (w + 63) / 64;
  std::vector<uint64_t> bits((size_t)h * n, 0);
  for (int y = 0; y < h; ++y)
    for (int x = 0; x < w; ++x)
      if (px[(size_t)y * w + x]) bits[(size_t)y * n + x / 64] |= 1ull << (x % 64);
  return bits;
}

void unpack_plane(const std::vector<uint64_t>& bits, int w, int h, uint8_t* px) {
  const int n = (w + 63) / 64;
  for (int y = 0; y < h; ++y)
    for (int x = 0; x < w; ++x) px[(size_t)y * w + x] = (uint8_t)((bits[(size_t)y * n + x / 64] >> (x % 64)) & 1);
}

std::vector<uint64_t> dilate_plane3(const std::vector<uint64_t>& bits, int w, int h) {
  const int n = (w + 63) / 64;
  const uint64_t last = (w & 63) ? ((1ull << (w & 63)) - 1ull) : ~0ull;
  std::vector<uint64_t> row((size_t)h * n), out((size_t)h * n);
  for (int y = 0; y < h; ++y)
    for (int i = 0; i < n; ++i) {
      const size_t k = (size_t)y * n + i;
      const uint64_t v = bits[k], prev = i > 0 ? bits[k - 1] : 0ull, next = i + 1 < n ? bits[k + 1] : 0ull;
      uint64_t acc = v | (v << 1) | (prev >> 63) | (v >> 1) | (next << 63);
      if (i == n - 1) acc &= last;
      row[k] = acc;
    }
  for (int y = 0; y < h; ++y)
    for (int i = 0; i < n; ++i) {
      const size_t k = (size_t)y * n + i;
      uint64_t acc = row[k];
      if (y > 0) acc |= row[k - n];
      if (y + 1 < h) acc |= row[k + n];
      out[k] = acc;
    }
  return out;
}

SlabStats grow_and_dilate_slabs(Comm& comm, SlabGrower& g, int w, int h, int depth, int z0, int z1, int connectivity,
                                int dilation) {
  const int rank = comm.rank(), n = comm.size();
  if (depth < n) throw std::runtime_error("z-slabs: volume depth " + std::to_string(depth) + " < " + std::to_string(n) +
                                          " ranks leaves empty slabs");
  const int d = z1 - z0;
  const size_t pw = plane_words(w, h), pbytes = pw * 8;
  const int below_rank = rank > 0 ? rank - 1 : -1, above_rank = rank + 1 < n ? rank + 1 : -1;
  SlabStats st;
  // ---- region growing: local fixpoints + boundary exchange until no rank adds a voxel ----------
  std::vector<uint64_t> nb_below(pw), nb_above(pw);
  for (bool first = true;; first = false) {
    st.sweeps += g.grow(first);
    ++st.rounds;
    const std::vector<uint64_t> top = g.region_plane(d - 1), bottom = g.region_plane(0);
    // My top plane goes up and the plane below my slab comes up from rank − 1; then the reverse.
    comm.sendrecv(top.data(), pbytes, above_rank, nb_below.data(), pbytes, below_rank);
    comm.sendrecv(bottom.data(), pbytes, below_rank, nb_above.data(), pbytes, above_rank);
    st.exchanged_bytes += (int64_t)((above_rank >= 0) + (below_rank >= 0)) * (int64_t)pbytes;
    int64_t added = 0;
    auto seed_from = [&](int zl, const std::vector<uint64_t>& nbp) {
      const std::vector<uint64_t> touch = connectivity == 26 ? dilate_plane3(nbp, w, h) : nbp;
      const std::vector<uint64_t> band = g.band_plane(zl), reg = g.region_plane(zl);
      std::vector<uint64_t> add(pw);
      int64_t k = 0;
      for (size_t i = 0; i < pw; ++i) {
        add[i] = band[i] & touch[i] & ~reg[i];
        k += __builtin_popcountll(add[i]);
      }
      if (k) g.or_region_plane(zl, add);
      added += k;
    };
    if (below_rank >= 0 && popcount(nb_below)) seed_from(0, nb_below);
    if (above_rank >= 0 && popcount(nb_above)) seed_from(d - 1, nb_above);
    comm.allreduce_sum_i64(&added, 1);
    if (added == 0) break;
  }
  // ---- cube dilation with r halo planes from each side -----------------------------------------
  const int r = dilation / 2;
  std::vector<std::vector<uint64_t>> below, above;
  if (r > 0) {
    const int rb = std::min(r, z0), ra = std::min(r, depth - z1);  // halo planes that exist
    if (depth / n >= r) {
      // Every slab holds ≥ r planes: the halo comes from the direct neighbours.
      std::vector<std::vector<uint64_t>> mine_top, mine_bottom;
      for (int k = std::max(0, d - r); k < d; ++k) mine_top.push_back(g.region_plane(k));
      for (int k = 0; k < std::min(r, d); ++k) mine_bottom.push_back(g.region_plane(k));
      const std::vector<uint8_t> tb = to_bytes(mine_top), bb = to_bytes(mine_bottom);
      std::vector<uint8_t> rb_buf((size_t)rb * pbytes), ra_buf((size_t)ra * pbytes);
      comm.sendrecv(tb.data(), above_rank >= 0 ? tb.size() : 0, above_rank, rb_buf.data(), rb_buf.size(), below_rank);
      comm.sendrecv(bb.data(), below_rank >= 0 ? bb.size() : 0, below_rank, ra_buf.data(), ra_buf.size(), above_rank);
      st.exchanged_bytes += (int64_t)(above_rank >= 0 ? tb.size() : 0) + (int64_t)(below_rank >= 0 ? bb.size() : 0);
      below = from_bytes(rb_buf.data(), (size_t)rb, pw);
      above = from_bytes(ra_buf.data(), (size_t)ra, pw);
    } else {
      // Thin slabs: the halo may span several ranks — every rank shares its first and last r planes.
      std::vector<std::vector<uint64_t>> ends;
      const int m = std::min(r, d);
      for (int k = 0; k < m; ++k) ends.push_back(g.region_plane(k));
      for (int k = d - m; k < d; ++k) ends.push_back(g.region_plane(k));
      const std::vector<uint8_t> mine = to_bytes(ends);
      st.exchanged_bytes += (int64_t)mine.size() * (n - 1);
      const auto all = comm.allgather_bytes(mine);
      auto plane_at = [&](int z) {
        for (int q = 0; q < n; ++q) {
          const auto [a, b] = slab_bounds(depth, q, n);
          if (z < a || z >= b) continue;
          const int dq = b - a, mq = std::min(r, dq);
          const int k = z - a < mq ? z - a : mq + (z - (b - mq));  // in q's first or last planes
          return from_bytes(all[(size_t)q].data() + (size_t)k * pbytes, 1, pw)[0];
        }
        throw std::runtime_error("z-slabs: halo plane without owner");
      };
      for (int z = z0 - rb; z < z0; ++z) below.push_back(plane_at(z));
      for (int z = z1; z < z1 + ra; ++z) above.push_back(plane_at(z));
    }
  }
  g.dilate(dilation, below, above);
  return st;
}

// ---- golden backend ------------------------------------------------------------------------------
GoldenSlabGrower::GoldenSlabGrower(std::vector<uint8_t> band, int w, int h, int d, std::vector<Seed> seeds,
                                   int connectivity)
    : band_(std::move(band)), region_(band_.size(), 0), w_(w), h_(h), d_(d), conn_(connectivity),
      seeds_(std::move(seeds)) {}

int GoldenSlabGrower::grow(bool first) {
  std::vector<Seed> s;
  if (first) {
    s = seeds_;
  } else {  // continue: every region voxel seeds the flood
    const size_t plane = (size_t)w_ * h_;
    for (size_t i = 0; i < region_.size(); ++i)
      if (region_[i]) s.push_back(Seed{(int32_t)(i % w_), (int32_t)((i % plane) / w_), (int32_t)(i / plane)});
  }
  region_ = golden::region_grow3d(band_, w_, h_, d_, s, conn_);
  return 1;
}

std::vector<uint64_t> GoldenSlabGrower::band_plane(int zl) { return pack_plane(&band_[(size_t)zl * w_ * h_], w_, h_); }
std::vector<uint64_t> GoldenSlabGrower::region_plane(int zl) {
  return pack_plane(&region_[(size_t)zl * w_ * h_], w_, h_);
}
void GoldenSlabGrower::or_region_plane(int zl, const std::vector<uint64_t>& bits) {
  std::vector<uint8_t> px((size_t)w_ * h_);
  unpack_plane(bits, w_, h_, px.data());
  uint8_t* r = &region_[(size_t)zl * w_ * h_];
  for (size_t i = 0; i < px.size(); ++i) r[i] |= px[i];
}

void GoldenSlabGrower::dilate(int size, const std::vector<std::vector<uint64_t>>& below,
                              const std::vector<std::vector<uint64_t>>& above) {
  const size_t plane = (size_t)w_ * h_;
  const int nb = (int)below.size(), na = (int)above.size();
  std::vector<uint8_t> ext(plane * (size_t)(nb + d_ + na));
  for (int k = 0; k < nb; ++k) unpack_plane(below[(size_t)k], w_, h_, &ext[(size_t)k * plane]);
  std::copy(region_.begin(), region_.end(), ext.begin() + (long)((size_t)nb * plane));
  for (int k = 0; k < na; ++k) unpack_plane(above[(size_t)k], w_, h_, &ext[(size_t)(nb + d_ + k) * plane]);
  const std::vector<uint8_t> dil = golden::dilate3d(ext, w_, h_, nb + d_ + na, size, ball);
  dilated_.assign(dil.begin() + (long)((size_t)nb * plane), dil.begin() + (long)((size_t)(nb + d_) * plane));
}

}  // namespace nm03
