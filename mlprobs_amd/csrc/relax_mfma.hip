// relax_mfma.hip -- evaluation variant of the consistency transform on the
// fp32 matrix cores (not the product path).
//
// P'_xy(i, j) = sum_z sum_k P_xz(i, k) P_zy(k, j) (CPNP/MSA.cpp:1172-1360) as
// dense 16x16 block products: every block image P(s, z) (rows = residues of
// s) is cut into 16x16 tiles, empty tiles dropped; output tile (I, J) of a
// pair's mask gathers sum_K A(I, K) C(J, K)^T over the K where both tiles of
// P(x, z) and P(y, z) are non-empty, with v_mfma_f32_16x16x4_f32.  The matrix
// cores accumulate with fused products (no rounding of a*b), so results
// differ from the reference's mul-then-add order in the last bits: this
// variant is held to the 1e-4 relative rule, never to
// bit identity, and only exists to measure the approach against
// k_relax_tile.  Rows ~9 entries wide spread over ~90 columns (C3) fill a
// 16x16 tile to a few percent, which is why the dense form loses.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cmath>
#include <string>
#include <thread>
#include <vector>

#include "../../include/mlpgpu.h"
#include "mlp_kernels.h"

namespace mlp {

typedef float f32x4 __attribute__((ext_vector_type(4)));

struct BlockImgs {
  const int32_t* grid;     // per image: nbr x nbc block indices (-1 = empty)
  const int16_t* krange;   // per image and block row: first, last non-empty K (first > last: none)
  const int64_t* goff;     // per (s index, z): offset of the image's grid
  const int64_t* roff;     // per (s index, z): offset of the image's krange rows
  const int32_t* nb;       // per sequence: blocks per side (ceil(L / 16))
  const float* blocks;     // 256 floats per block, row-major
};
struct MfmaOut {
  const int32_t* ox;       // per output: s index of x, of y, first tile, tile count
  const int32_t* oy;
  const int32_t* tfirst;
  const int32_t* tcount;
  const int32_t* tiles;    // I | J << 16
  const int32_t* xseq;     // per output: sequence number of x, of y
  const int32_t* yseq;
  float* out;              // 256 floats per tile (row-major)
  int n, nsets;
};

constexpr int kMfmaTiles = 8;  // output tiles per wave pass (4 accumulator VGPRs each)

__global__ __launch_bounds__(256) void k_relax_blockmfma(BlockImgs B, MfmaOut O) {
  const int o = blockIdx.x;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int sx = O.ox[o], sy = O.oy[o], x = O.xseq[o], y = O.yseq[o];
  const int t0 = O.tfirst[o], nt = O.tcount[o];
  // lane l holds row l & 15, columns 4 (l >> 4) .. + 3 of a block: k-slice q
  // of the four MFMAs takes column 4 (l >> 4) + q of both operands
  const int frag = (lane & 15) * 16 + 4 * (lane >> 4);
  for (int base = wave * kMfmaTiles; base < nt; base += 4 * kMfmaTiles) {
    f32x4 acc[kMfmaTiles];
    int I[kMfmaTiles], J[kMfmaTiles];
#pragma unroll
    for (int t = 0; t < kMfmaTiles; ++t) {
      acc[t] = f32x4{0.f, 0.f, 0.f, 0.f};
      const int tt = base + t < nt ? O.tiles[t0 + base + t] : -1;
      I[t] = tt < 0 ? -1 : (tt & 0xffff);
      J[t] = tt < 0 ? -1 : (tt >> 16);
    }
    for (int z = 0; z < O.n; ++z) {
      if (z == x || z == y) continue;
      const int64_t ga = B.goff[(int64_t)sx * O.n + z], gc = B.goff[(int64_t)sy * O.n + z];
      const int16_t* ra = B.krange + 2 * B.roff[(int64_t)sx * O.n + z];
      const int16_t* rc = B.krange + 2 * B.roff[(int64_t)sy * O.n + z];
      const int nbc = B.nb[z];
#pragma unroll
      for (int t = 0; t < kMfmaTiles; ++t) {
        if (I[t] < 0) continue;
        const int k0 = max((int)ra[2 * I[t]], (int)rc[2 * J[t]]);
        const int k1 = min((int)ra[2 * I[t] + 1], (int)rc[2 * J[t] + 1]);
        for (int K = k0; K <= k1; ++K) {
          const int ia = B.grid[ga + (int64_t)I[t] * nbc + K], ic = B.grid[gc + (int64_t)J[t] * nbc + K];
          if (ia < 0 || ic < 0) continue;
          const float4 a = *reinterpret_cast<const float4*>(B.blocks + (int64_t)ia * 256 + frag);
          const float4 c = *reinterpret_cast<const float4*>(B.blocks + (int64_t)ic * 256 + frag);
          acc[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(a.x, c.x, acc[t], 0, 0, 0);
          acc[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(a.y, c.y, acc[t], 0, 0, 0);
          acc[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(a.z, c.z, acc[t], 0, 0, 0);
          acc[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(a.w, c.w, acc[t], 0, 0, 0);
        }
      }
    }
    // D: column lane & 15, row 4 (lane >> 4) + r
#pragma unroll
    for (int t = 0; t < kMfmaTiles; ++t) {
      if (I[t] < 0) continue;
      float* dst = O.out + (int64_t)(t0 + base + t) * 256;
#pragma unroll
      for (int r = 0; r < 4; ++r) dst[(4 * (lane >> 4) + r) * 16 + (lane & 15)] = acc[t][r];
    }
  }
}

// Host driver: blocks of every image P(s, z), s in xs or ys, from the
// exported canonical store; outputs (x, y), x in xs, y in ys, x < y.
int relax_blockmfma_eval(int n, const int32_t* lens, const int64_t* rp_off, const int32_t* rowptr,
                         const int64_t* ent_off, const uint16_t* cols, const float* vals, int nx, const int32_t* xs,
                         int ny, const int32_t* ys, double* res, std::string& err) {
  auto pidx = [n](int a, int b) -> int64_t {  // a < b
    return (int64_t)a * (2 * (int64_t)n - a - 1) / 2 + (b - a - 1);
  };
  std::vector<int> sets;
  for (int k = 0; k < nx; k++) sets.push_back(xs[k]);
  for (int k = 0; k < ny; k++) sets.push_back(ys[k]);
  const int ns = (int)sets.size();
  std::vector<int32_t> nb(n);
  for (int s = 0; s < n; s++) nb[s] = (lens[s] + 15) / 16;
  // per image: grid offset (entries) and krange row offset
  std::vector<int64_t> goff((size_t)ns * n, 0);
  int64_t gtot = 0;
  for (int si = 0; si < ns; si++)
    for (int z = 0; z < n; z++) {
      goff[(size_t)si * n + z] = gtot;
      if (z != sets[si]) gtot += (int64_t)nb[sets[si]] * nb[z];
    }
  std::vector<int32_t> grid(std::max<int64_t>(gtot, 1), -1);
  std::vector<int64_t> roff((size_t)ns * n, 0);
  int64_t rtot = 0;
  for (int si = 0; si < ns; si++)
    for (int z = 0; z < n; z++) {
      roff[(size_t)si * n + z] = rtot;
      if (z != sets[si]) rtot += nb[sets[si]];
    }
  // blocks, built per image in parallel (block ids assigned per image, then rebased)
  struct Img { std::vector<float> blk; std::vector<int32_t> g; std::vector<int16_t> kr; };
  std::vector<Img> imgs((size_t)ns * n);
  std::atomic<int64_t> next{0};
  auto build = [&]() {
    for (int64_t q; (q = next.fetch_add(1)) < (int64_t)ns * n;) {
      const int si = (int)(q / n), z = (int)(q % n), s = sets[si];
      if (z == s) continue;
      Img& im = imgs[q];
      const int nr = nb[s], nc = nb[z];
      im.g.assign((size_t)nr * nc, -1);
      im.kr.assign((size_t)2 * nr, 0);
      for (int r = 0; r < nr; r++) { im.kr[2 * r] = (int16_t)nc; im.kr[2 * r + 1] = -1; }
      auto put = [&](int i, int k, float v) {  // 1-based residues of s and z
        const int bi = (i - 1) >> 4, bk = (k - 1) >> 4;
        int32_t& id = im.g[(size_t)bi * nc + bk];
        if (id < 0) {
          id = (int32_t)(im.blk.size() / 256);
          im.blk.resize(im.blk.size() + 256, 0.f);
        }
        im.blk[(size_t)id * 256 + ((i - 1) & 15) * 16 + ((k - 1) & 15)] = v;
        im.kr[2 * bi] = (int16_t)std::min<int>(im.kr[2 * bi], bk);
        im.kr[2 * bi + 1] = (int16_t)std::max<int>(im.kr[2 * bi + 1], bk);
      };
      if (s < z) {
        const int64_t p = pidx(s, z);
        const int32_t* rp = rowptr + rp_off[p];
        for (int i = 1; i <= lens[s]; i++)
          for (int e = rp[i]; e < rp[i + 1]; e++) put(i, cols[ent_off[p] + e], vals[ent_off[p] + e]);
      } else {
        const int64_t p = pidx(z, s);
        const int32_t* rp = rowptr + rp_off[p];
        for (int r = 1; r <= lens[z]; r++)
          for (int e = rp[r]; e < rp[r + 1]; e++) put(cols[ent_off[p] + e], r, vals[ent_off[p] + e]);
      }
    }
  };
  {
    const int nth = std::max(1, std::min(16, (int)std::thread::hardware_concurrency()));
    std::vector<std::thread> th;
    for (int w = 0; w < nth; w++) th.emplace_back(build);
    for (auto& t : th) t.join();
  }
  int64_t nblocks = 0;
  std::vector<int16_t> krange((size_t)std::max<int64_t>(2 * rtot, 2), 0);
  for (int64_t q = 0; q < (int64_t)ns * n; q++) {
    const Img& im = imgs[q];
    if (im.g.empty()) continue;
    for (size_t k = 0; k < im.g.size(); k++) grid[goff[q] + k] = im.g[k] < 0 ? -1 : (int32_t)(im.g[k] + nblocks);
    std::copy(im.kr.begin(), im.kr.end(), krange.begin() + 2 * roff[q]);
    nblocks += (int64_t)im.blk.size() / 256;
  }
  std::vector<float> blocks((size_t)std::max<int64_t>(nblocks, 1) * 256);
  for (int64_t q = 0, at = 0; q < (int64_t)ns * n; q++) {
    const Img& im = imgs[q];
    std::copy(im.blk.begin(), im.blk.end(), blocks.begin() + at);
    at += (int64_t)im.blk.size();
  }
  imgs.clear();
  imgs.shrink_to_fit();
  // outputs and their mask tiles
  std::vector<int32_t> ox, oy, xq, yq, tfirst, tcount, tiles;
  double dense_macs = 0;
  for (int a = 0; a < nx; a++)
    for (int b = 0; b < ny; b++) {
      const int x = xs[a], y = ys[b];
      if (x >= y) continue;
      const int64_t p = pidx(x, y);
      const int32_t* rp = rowptr + rp_off[p];
      std::vector<int32_t> t;
      for (int i = 1; i <= lens[x]; i++)
        for (int e = rp[i]; e < rp[i + 1]; e++) t.push_back(((i - 1) >> 4) | (((int)cols[ent_off[p] + e] - 1) >> 4) << 16);
      std::sort(t.begin(), t.end());
      t.erase(std::unique(t.begin(), t.end()), t.end());
      ox.push_back(a);
      oy.push_back(nx + b);
      xq.push_back(x);
      yq.push_back(y);
      tfirst.push_back((int32_t)tiles.size());
      tcount.push_back((int32_t)t.size());
      tiles.insert(tiles.end(), t.begin(), t.end());
      // dense MACs: block products the kernel issues
      for (int32_t tt : t) {
        const int I = tt & 0xffff, J = tt >> 16;
        for (int z = 0; z < n; z++) {
          if (z == x || z == y) continue;
          const int64_t qa = (int64_t)a * n + z, qc = (int64_t)(nx + b) * n + z;
          const int nc = nb[z];
          for (int K = 0; K < nc; K++)
            if (grid[goff[qa] + (int64_t)I * nc + K] >= 0 && grid[goff[qc] + (int64_t)J * nc + K] >= 0) dense_macs += 4096;
        }
      }
    }
  const int nout = (int)ox.size();
  if (!nout) {
    err = "blockmfma eval: no outputs (need x < y)";
    return MLP_ERR_ARG;
  }
  // device buffers
  auto up = [&](const void* h, size_t bytes, void** d) -> bool {
    if (hipMalloc(d, std::max<size_t>(bytes, 16)) != hipSuccess) return false;
    return hipMemcpy(*d, h, bytes, hipMemcpyHostToDevice) == hipSuccess;
  };
  void *d_grid = nullptr, *d_kr = nullptr, *d_goff = nullptr, *d_roff = nullptr, *d_nb = nullptr, *d_blk = nullptr, *d_ox = nullptr,
       *d_oy = nullptr, *d_tf = nullptr, *d_tc = nullptr, *d_t = nullptr, *d_xq = nullptr, *d_yq = nullptr,
       *d_out = nullptr;
  bool ok = up(grid.data(), grid.size() * 4, &d_grid) && up(krange.data(), krange.size() * 2, &d_kr) &&
            up(goff.data(), goff.size() * 8, &d_goff) && up(roff.data(), roff.size() * 8, &d_roff) && up(nb.data(), nb.size() * 4, &d_nb) &&
            up(blocks.data(), blocks.size() * 4, &d_blk) && up(ox.data(), ox.size() * 4, &d_ox) &&
            up(oy.data(), oy.size() * 4, &d_oy) && up(tfirst.data(), tfirst.size() * 4, &d_tf) &&
            up(tcount.data(), tcount.size() * 4, &d_tc) && up(tiles.data(), tiles.size() * 4, &d_t) &&
            up(xq.data(), xq.size() * 4, &d_xq) && up(yq.data(), yq.size() * 4, &d_yq) &&
            hipMalloc(&d_out, tiles.size() * 256 * 4) == hipSuccess;
  double secs = 0;
  std::vector<float> out(tiles.size() * 256);
  if (ok) {
    BlockImgs B{(const int32_t*)d_grid, (const int16_t*)d_kr, (const int64_t*)d_goff, (const int64_t*)d_roff,
                (const int32_t*)d_nb, (const float*)d_blk};
    MfmaOut O{(const int32_t*)d_ox, (const int32_t*)d_oy, (const int32_t*)d_tf, (const int32_t*)d_tc,
              (const int32_t*)d_t, (const int32_t*)d_xq, (const int32_t*)d_yq, (float*)d_out, n, ns};
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    hipLaunchKernelGGL(k_relax_blockmfma, dim3(nout), dim3(256), 0, 0, B, O);  // warm-up
    hipEventRecord(e0, 0);
    hipLaunchKernelGGL(k_relax_blockmfma, dim3(nout), dim3(256), 0, 0, B, O);
    hipEventRecord(e1, 0);
    ok = hipEventSynchronize(e1) == hipSuccess && hipGetLastError() == hipSuccess;
    float ms = 0;
    hipEventElapsedTime(&ms, e0, e1);
    secs = ms * 1e-3;
    hipEventDestroy(e0);
    hipEventDestroy(e1);
    ok = ok && hipMemcpy(out.data(), d_out, out.size() * 4, hipMemcpyDeviceToHost) == hipSuccess;
  }
  for (void* d : {d_grid, d_kr, d_goff, d_roff, d_nb, d_blk, d_ox, d_oy, d_tf, d_tc, d_t, d_xq, d_yq, d_out})
    if (d) hipFree(d);
  if (!ok) {
    err = "blockmfma eval: device error";
    return MLP_ERR_HIP;
  }
  // the same sums in double on the host, from the blocks, on a strided
  // sample of each output's mask cells
  double max_rel = 0;
  int64_t cells = 0;
  for (int o = 0; o < nout; o++) {
    const int x = xq[o], y = yq[o];
    const int64_t p = pidx(x, y);
    const int32_t* rp = rowptr + rp_off[p];
    int64_t k = 0;
    for (int i = 1; i <= lens[x]; i++)
      for (int e = rp[i]; e < rp[i + 1]; e++, k++) {
        if (k % (nout > 256 ? 127 : 17)) continue;
        const int j = cols[ent_off[p] + e];
        const int I = (i - 1) >> 4, J = (j - 1) >> 4;
        double sum = 0;
        for (int z = 0; z < n; z++) {
          if (z == x || z == y) continue;
          const int64_t qa = (int64_t)ox[o] * n + z, qc = (int64_t)oy[o] * n + z;
          const int nc = nb[z];
          for (int K = 0; K < nc; K++) {
            const int32_t ia = grid[goff[qa] + (int64_t)I * nc + K], ic = grid[goff[qc] + (int64_t)J * nc + K];
            if (ia < 0 || ic < 0) continue;
            const float* A = &blocks[(size_t)ia * 256 + ((i - 1) & 15) * 16];
            const float* C = &blocks[(size_t)ic * 256 + ((j - 1) & 15) * 16];
            for (int kk = 0; kk < 16; kk++) sum += (double)A[kk] * C[kk];
          }
        }
        const int32_t key = I | J << 16;
        const auto it = std::lower_bound(tiles.begin() + tfirst[o], tiles.begin() + tfirst[o] + tcount[o], key);
        const float got = out[(size_t)(it - tiles.begin()) * 256 + ((i - 1) & 15) * 16 + ((j - 1) & 15)];
        if (sum > 0) max_rel = std::max(max_rel, std::fabs(got - sum) / sum);
        cells++;
      }
  }
  res[0] = secs;
  res[1] = dense_macs;
  res[2] = (double)nout;
  res[3] = max_rel;
  res[4] = (double)cells;
  res[5] = (double)tiles.size();
  res[6] = (double)nblocks;
  return MLP_OK;
}

}  // namespace mlp
