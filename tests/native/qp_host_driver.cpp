// Test driver for the host stages of the quickprobs drop-in
// (mlprobs_amd/cli/qp_host.cpp).  CPU only; the CPU oracle supplies what the
// GPU computes in the real binary (tests/test_cli_host.py):
//   qp_host_driver tree IN OUT   IN: n, D (n x n f32) -> OUT: weights (n f32),
//                                subtree distances (n x n f32)
//   qp_host_driver align IN      IN: n, refinement, then per sequence
//                                (header, residues), D (n x n f32), the
//                                consistency-transformed sparse set (row_ptr
//                                i32, ent_off i64, cols u16, vals f32)
//                                -> the FASTA of construction + refinement.
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <string>
#include <vector>

#include <random>

#include "msa_host.h"
#include "qp_host.h"

template <class T>
static void rd(FILE* f, T* p, size_t n) {
  if (n && fread(p, sizeof(T), n, f) != n) { fprintf(stderr, "short read\n"); exit(2); }
}

int main(int argc, char** argv) {
  if (argc < 3) return 2;
  if (!strcmp(argv[1], "mea") && argc == 5) {  // threaded (wave) vs serial MEA on a random matrix
    const int L1 = atoi(argv[3]), L2 = atoi(argv[4]);
    std::mt19937 g((unsigned)atoi(argv[2]));
    std::uniform_real_distribution<float> u(0.f, 1.f);
    std::vector<float> post((size_t)(L1 + 1) * (L2 + 1));
    for (float& x : post) x = u(g) < 0.9f ? 0.f : u(g);  // sparse-ish, with ties
    float s1 = 0, s2 = 0;
    const std::string a = cpnp::mea_path_serial(L1, L2, post.data(), &s1);
    const std::string b = cpnp::mea_path_wave(L1, L2, post.data(), &s2);
    printf("%s\n", (a == b && s1 == s2) ? "same" : "DIFF");
    return 0;
  }
  FILE* f = fopen(argv[2], "rb");
  if (!f) return 2;
  if (!strcmp(argv[1], "tree")) {
    int32_t n;
    rd(f, &n, 1);
    std::vector<float> D((size_t)n * n);
    rd(f, D.data(), D.size());
    fclose(f);
    const qph::Tree t = qph::build_tree(D, n);
    const std::vector<float> s = t.subtree_distances();
    FILE* o = fopen(argv[3], "wb");
    fwrite(t.weights.data(), sizeof(float), n, o);
    fwrite(s.data(), sizeof(float), s.size(), o);
    fclose(o);
    return 0;
  }
  int32_t hdr[2];
  rd(f, hdr, 2);
  const int n = hdr[0];
  qph::Options opt;
  opt.refinement = hdr[1];
  std::vector<qph::Seq> seqs(n);
  for (int k = 0; k < n; k++) {
    int32_t len;
    rd(f, &len, 1);
    seqs[k].header.resize(len);
    rd(f, &seqs[k].header[0], len);
    rd(f, &len, 1);
    std::string s(len, ' ');
    rd(f, &s[0], len);
    seqs[k].data = "@" + s;
    seqs[k].label = seqs[k].sort_label = k;
  }
  std::vector<float> D((size_t)n * n);
  rd(f, D.data(), D.size());
  qph::Sparse sp;
  sp.n = n;
  for (auto& r : seqs) sp.lens.push_back(r.length());
  const int64_t P = (int64_t)n * (n - 1) / 2;
  sp.rp_off.assign(P + 1, 0);
  for (int a = 0, p = 0; a < n; a++)
    for (int b = a + 1; b < n; b++, p++) sp.rp_off[p + 1] = sp.rp_off[p] + sp.lens[a] + 2;
  sp.row_ptr.resize(sp.rp_off[P]);
  sp.ent_off.resize(P + 1);
  rd(f, sp.row_ptr.data(), sp.row_ptr.size());
  rd(f, sp.ent_off.data(), P + 1);
  sp.cols.resize(sp.ent_off[P] + 1);
  sp.vals.resize(sp.ent_off[P] + 1);
  rd(f, sp.cols.data(), sp.ent_off[P]);
  rd(f, sp.vals.data(), sp.ent_off[P]);
  fclose(f);
  sp.build_views();
  const qph::Tree tree = qph::build_tree(D, n);
  qph::PosteriorBackend be;
  be.host_sparse = [&]() -> const qph::Sparse& { return sp; };
  const qph::Profile aln = qph::construct_and_refine(seqs, be, tree, opt, 4);
  std::string out;
  qph::write_fasta(out, aln);
  fwrite(out.data(), 1, out.size(), stdout);
  return 0;
}
