// Test driver for the host stages of the c_p_np_aln drop-in
// (mlprobs_amd/cli/msa_host.cpp): reads the family, distances and the
// consistency-transformed sparse set from a binary file (written by
// tests/test_cli_host.py from the CPU oracle) and prints the MFA that
// tree + progressive alignment + refinement produce (header flag bit 1: the
// -p 1 stages instead, alignment graph + refinement).  CPU only.
#include <stdio.h>
#include <stdlib.h>

#include <string>
#include <vector>

#include "msa_host.h"

template <class T>
static void rd(FILE* f, T* p, size_t n) {
  if (n && fread(p, sizeof(T), n, f) != n) { fprintf(stderr, "short read\n"); exit(2); }
}

int main(int argc, char** argv) {
  if (argc < 2) return 2;
  FILE* f = fopen(argv[1], "rb");
  if (!f) return 2;
  int32_t hdr[5];
  rd(f, hdr, 5);
  const int n = hdr[0], pid = hdr[1], vpid = hdr[2];
  cpnp::Options opt;
  opt.refinement = hdr[3];
  opt.align_order = (hdr[4] & 1) != 0;
  const bool np = (hdr[4] & 2) != 0;
  std::vector<cpnp::Row> seqs(n);
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
  std::vector<std::vector<float>> D(n, std::vector<float>(n));
  for (int a = 0; a < n; a++) rd(f, D[a].data(), n);
  cpnp::SparseSet sp;
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
  cpnp::Profile aln;
  if (np) {
    aln = cpnp::np_refinement(cpnp::graph_alignment(seqs, sp), sp, D, opt);
  } else {
    const cpnp::GuideTree tree = cpnp::build_tree(D, vpid);
    aln = cpnp::progressive_alignment(seqs, sp, tree, pid, opt);
  }
  std::string out;
  cpnp::write_mfa(out, aln);
  fwrite(out.data(), 1, out.size(), stdout);
  return 0;
}
