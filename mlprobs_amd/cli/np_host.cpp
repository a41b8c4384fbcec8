// np_host.cpp -- host stages of the non-progressive strategy (c_p_np_aln -p 1,
// MSA::npdoAlign, CPNP/MSA.cpp:1084-1140) after the GPU posteriors and
// consistency rounds: the alignment graph (ComputeGraph + AlignGraph,
// CPNP/MSA.cpp:1776-1844, CPNP/AlignGraph.h) and its refinement
// (DoRefinement + FindSimilar, CPNP/MSA.cpp:1852-2082).
//
// The graph is the reference's, decision for decision: residue pairs are
// visited in the order of the reference's own quicksort of the posteriors
// (ties fall where its partition scheme puts them), and each pair creates a
// column, extends one or merges two under the same cycle tests and edge
// removals, so the child lists (whose order drives the depth-first path) end
// up identical.  Only the data structures differ: ancestor / descendant sets
// are word bitsets updated in place instead of vector<bool> copies, the graph
// is edited in place instead of through a full copy per pair, residue ->
// column lookups go through per-sequence ordered sets, and the path is a
// linked list.
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include <algorithm>
#include <cmath>
#include <set>

#include "msa_host.h"

namespace cpnp {

namespace {

// AlignGraph::Partition / Quick_sort (AlignGraph.h:62-112): ascending, with
// the reference's hole-filling partition around arr[low] (the single-thread
// branch the constructor always takes: omp_get_num_threads() is 1 outside a
// parallel region, AlignGraph.h:913-917).  Disjoint subranges are sorted
// independently, so an explicit stack gives the recursive result.
int partition(int low, int high, float* arr, int* ind) {
  const float pivot = arr[low];
  const int ip = ind[low];
  while (high > low) {
    float hv = arr[high];
    int ih = ind[high];
    while (pivot <= hv) {
      if (high <= low) break;
      --high;
      hv = arr[high];
      ih = ind[high];
    }
    arr[low] = hv;
    ind[low] = ih;
    float lv = arr[low];
    int il = ind[low];
    while (pivot >= lv) {
      if (high <= low) break;
      ++low;
      lv = arr[low];
      il = ind[low];
    }
    arr[high] = lv;
    ind[high] = il;
  }
  arr[low] = pivot;
  ind[low] = ip;
  return low;
}

void quick_sort(std::vector<float>& a, std::vector<int>& ind) {
  std::vector<std::pair<int, int>> todo;
  if (a.size() > 1) todo.push_back({0, (int)a.size() - 1});
  while (!todo.empty()) {
    const auto [lo, hi] = todo.back();
    todo.pop_back();
    if (lo >= hi) continue;
    const int p = partition(lo, hi, a.data(), ind.data());
    todo.push_back({p + 1, hi});
    todo.push_back({lo, p - 1});
  }
}

// Rows of bits over node indices (the reference's Ancs / Descs,
// SafeVector<SafeVector<bool>>), kept at a common word stride.
struct BitRows {
  int words = 0;
  std::vector<uint64_t> w;
  uint64_t* row(int r) { return w.data() + (size_t)r * words; }
  const uint64_t* row(int r) const { return w.data() + (size_t)r * words; }
  bool test(int r, int b) const { return (row(r)[b >> 6] >> (b & 63)) & 1; }
  void set(int r, int b) { row(r)[b >> 6] |= 1ull << (b & 63); }
  void reserve_bits(int nrows, int bits) {  // keep every row able to hold `bits`
    const int need = (bits + 63) / 64;
    if (need <= words) return;
    const int nw = std::max(need, words * 2 + 1);
    std::vector<uint64_t> x((size_t)nrows * nw, 0);
    for (int r = 0; r < nrows; r++) memcpy(x.data() + (size_t)r * nw, row(r), sizeof(uint64_t) * words);
    w.swap(x);
    words = nw;
  }
  int push_zero() {
    w.resize(w.size() + words, 0);
    return (int)(w.size() / words) - 1;
  }
  void or_into(int dst, const uint64_t* src) {
    uint64_t* d = row(dst);
    for (int k = 0; k < words; k++) d[k] |= src[k];
  }
  // AlignGraph::Update(SafeVector<bool>, cy, msize): bit cy leaves, the bits
  // above it move down one (bits at or above the node count are always 0)
  static void drop_bit(uint64_t* x, int nw, int cy) {
    const int k = cy >> 6, b = cy & 63;
    const uint64_t keep = b ? ((1ull << b) - 1) : 0;
    const uint64_t above = b == 63 ? 0 : (x[k] >> (b + 1)) << b;
    x[k] = (x[k] & keep) | above | ((k + 1 < nw ? (x[k + 1] & 1) : 0) << 63);
    for (int t = k + 1; t < nw; t++) x[t] = (x[t] >> 1) | ((t + 1 < nw ? (x[t + 1] & 1) : 0) << 63);
  }
  void erase_row(int r, int nrows) {
    memmove(row(r), row(r + 1), sizeof(uint64_t) * words * (size_t)(nrows - r - 1));
    w.resize((size_t)(nrows - 1) * words);
  }
};

template <class F>
void for_bits(const uint64_t* x, int nbits, F f) {
  const int nw = (nbits + 63) / 64;
  for (int k = 0; k < nw; k++) {
    uint64_t v = x[k];
    if (k == nw - 1 && (nbits & 63)) v &= (1ull << (nbits & 63)) - 1;
    while (v) {
      const int b = __builtin_ctzll(v);
      f(k * 64 + b);
      v &= v - 1;
    }
  }
}

bool has(const std::vector<int>& v, int x) { return std::find(v.begin(), v.end(), x) != v.end(); }
void remove_all(std::vector<int>& v, int x) { v.erase(std::remove(v.begin(), v.end(), x), v.end()); }
void push_unique(std::vector<int>& v, int x) {   // AlignGraph::Union_VI of one element
  if (!has(v, x)) v.push_back(x);
}

struct Graph {
  int nseq = 0, maxlen = 0;
  std::vector<std::vector<int>> G;          // G[i]: children of node i, in order
  BitRows anc, desc;                        // anc.test(i, j): j is an ancestor of i
  // residue placement: stable node ids (a node keeps its id while its index
  // shifts down when an earlier-indexed merge removes a node before it)
  std::vector<std::vector<int>> present;    // present[s][r]: node id or -1
  std::vector<std::set<int>> placed;        // placed[s]: residues r of s in some node
  std::vector<int> idx_of;                  // node id -> index
  std::vector<int> id_of;                   // index -> node id
  std::vector<std::vector<std::pair<int, int>>> members;  // per node id: (seq, residue)
  std::vector<std::vector<uint64_t>> seqbits;              // per node id: sequences present

  int node_at(int s, int r) const { return present[s][r] < 0 ? -1 : idx_of[present[s][r]]; }
  bool node_has_seq(int node, int s) const {
    const std::vector<uint64_t>& b = seqbits[id_of[node]];
    return (b[s >> 6] >> (s & 63)) & 1;
  }
  void place(int s, int r, int node) {
    const int id = id_of[node];
    present[s][r] = id;
    placed[s].insert(r);
    members[id].push_back({s, r});
    seqbits[id][s >> 6] |= 1ull << (s & 63);
  }
  int new_id(int index) {
    const int id = (int)members.size();
    members.emplace_back();
    seqbits.emplace_back((nseq + 63) / 64, 0);
    idx_of.push_back(index);
    return id;
  }

  // AlignGraph::FindCloseNodes (AlignGraph.h:187-221): the nodes of the
  // nearest placed residues before and after (s, r); "after" is searched up
  // to maxlength and ignores a hit at position 10000 (the reference's inf)
  void close_nodes(int s, int r, std::vector<int>& par, std::vector<int>& chi) const {
    par.clear();
    chi.clear();
    const std::set<int>& pl = placed[s];
    auto it = pl.lower_bound(r);
    if (it != pl.begin()) par.push_back(node_at(s, *std::prev(it)));
    auto jt = pl.upper_bound(r);
    if (jt != pl.end() && *jt < maxlen && *jt != 10000) chi.push_back(node_at(s, *jt));
  }
  // ancestors / descendants closure after node `at` gained ancestors AA and
  // descendants DD (AlignGraph.h:470-485, 585-601, 736-751)
  void close_sets(int at, const std::vector<uint64_t>& A, const std::vector<uint64_t>& D, int n) {
    std::vector<int> AA, DD;
    for_bits(A.data(), n, [&](int j) { AA.push_back(j); });
    for_bits(D.data(), n, [&](int j) { DD.push_back(j); });
    for (int d : DD) {
      anc.set(d, at);
      anc.or_into(d, A.data());
    }
    for (int a : AA) {
      desc.or_into(a, D.data());
      desc.set(a, at);
    }
  }

  // AlignGraph::CheckAddNewNode (AlignGraph.h:381-488)
  bool add_node(int xs, int xr, int ys, int yr) {
    std::vector<int> sx0, sx1, sy0, sy1;
    close_nodes(xs, xr, sx0, sx1);
    close_nodes(ys, yr, sy0, sy1);
    std::vector<int> parent = sx0, child = sx1;
    for (int v : sy0) push_unique(parent, v);
    for (int v : sy1) push_unique(child, v);
    bool ok = true;
    if (sx0.size() == 1 && sy1.size() == 1) ok = ok && !desc.test(sy1[0], sx0[0]) && sx0[0] != sy1[0];
    if (sy0.size() == 1 && sx1.size() == 1) ok = ok && !desc.test(sx1[0], sy0[0]) && sy0[0] != sx1[0];
    if (!ok) return false;
    const int n = (int)G.size();  // the new node's index
    // redundant-edge tests read the sets before the new node exists
    const bool rm_x0 = sx0.size() == 1 && sy0.size() == 1 && desc.test(sx0[0], sy0[0]);
    const bool rm_y0 = sx0.size() == 1 && sy0.size() == 1 && desc.test(sy0[0], sx0[0]);
    const bool rm_cy = sx1.size() == 1 && sy1.size() == 1 && desc.test(sx1[0], sy1[0]);
    const bool rm_cx = sx1.size() == 1 && sy1.size() == 1 && desc.test(sy1[0], sx1[0]);
    G.push_back(child);
    for (int p : parent) G[p].push_back(n);
    if (rm_x0) remove_all(G[sx0[0]], n);
    if (rm_y0) remove_all(G[sy0[0]], n);
    if (rm_cy) remove_all(G[n], sy1[0]);
    if (rm_cx) remove_all(G[n], sx1[0]);
    for (int p : parent)
      for (int c : child) remove_all(G[p], c);
    id_of.push_back(new_id(n));
    place(xs, xr, n);
    place(ys, yr, n);
    const int gsz = n + 1;
    anc.reserve_bits(n, gsz + 1);
    desc.reserve_bits(n, gsz + 1);
    std::vector<uint64_t> A(anc.words, 0), D(desc.words, 0);
    if (!parent.empty()) memcpy(A.data(), anc.row(parent[0]), sizeof(uint64_t) * anc.words);
    if (parent.size() == 2)
      for_bits(anc.row(parent[1]), gsz - 1, [&](int j) { A[j >> 6] |= 1ull << (j & 63); });
    for (int p : parent) A[p >> 6] |= 1ull << (p & 63);
    if (!child.empty()) memcpy(D.data(), desc.row(child[0]), sizeof(uint64_t) * desc.words);
    if (child.size() == 2)
      for_bits(desc.row(child[1]), gsz - 1, [&](int j) { D[j >> 6] |= 1ull << (j & 63); });
    for (int c : child) D[c >> 6] |= 1ull << (c & 63);
    const int ra = anc.push_zero(), rd = desc.push_zero();
    memcpy(anc.row(ra), A.data(), sizeof(uint64_t) * anc.words);
    memcpy(desc.row(rd), D.data(), sizeof(uint64_t) * desc.words);
    close_sets(n, A, D, gsz);
    return true;
  }

  // AlignGraph::CheckAddColumnEx (AlignGraph.h:497-605): residue y joins node cx
  bool extend(int ys, int yr, int cx) {
    std::vector<int> par, chi;
    close_nodes(ys, yr, par, chi);
    bool ok = true;
    if (!chi.empty()) ok = !desc.test(chi[0], cx) && chi[0] != cx;
    if (!par.empty()) ok = ok && !desc.test(cx, par[0]) && par[0] != cx;
    if (!ok) return false;
    const bool rm_p = par.size() == 1 && desc.test(par[0], cx) && !has(G[par[0]], cx);
    const bool rm_c = chi.size() == 1 && desc.test(cx, chi[0]) && !has(G[cx], chi[0]);
    for (int p : par) push_unique(G[p], cx);
    for (int c : chi) push_unique(G[cx], c);
    if (rm_p) remove_all(G[par[0]], cx);
    if (rm_c) remove_all(G[cx], chi[0]);
    if (par.size() == 1 && chi.size() == 1) remove_all(G[par[0]], chi[0]);
    place(ys, yr, cx);
    const int gsz = (int)G.size();
    std::vector<uint64_t> A(anc.words, 0), D(desc.words, 0);
    if (!par.empty()) memcpy(A.data(), anc.row(par[0]), sizeof(uint64_t) * anc.words);
    for (int p : par) A[p >> 6] |= 1ull << (p & 63);
    if (!chi.empty()) memcpy(D.data(), desc.row(chi[0]), sizeof(uint64_t) * desc.words);
    for (int c : chi) D[c >> 6] |= 1ull << (c & 63);
    for_bits(A.data(), gsz, [&](int j) { anc.set(cx, j); });
    for_bits(D.data(), gsz, [&](int j) { desc.set(cx, j); });
    std::vector<uint64_t> AC(anc.row(cx), anc.row(cx) + anc.words), DC(desc.row(cx), desc.row(cx) + desc.words);
    close_sets(cx, AC, DC, gsz);
    return true;
  }

  // AlignGraph::CheckAddColumnMrg (AlignGraph.h:614-755): node cy (> cx)
  // merges into cx; nodes above cy shift down one index
  bool merge(int cx, int cy) {
    if (desc.test(cx, cy) || desc.test(cy, cx)) return false;
    const int n = (int)G.size();
    auto U = [&](int i) { return i < cy ? i : i == cy ? cx : i - 1; };
    // the renumbered graph (AlignGraph.h:620-646)
    std::vector<int> child_x = G[cx];
    for (int v : G[cy]) push_unique(child_x, v);
    std::vector<std::vector<int>> T;
    T.reserve(n - 1);
    for (int j = 0; j < n; j++) {
      if (j == cx) {
        std::vector<int> ch;
        for (int v : child_x) ch.push_back(U(v));
        T.push_back(std::move(ch));
      } else if (j != cy) {
        std::vector<int> nodes;
        bool flag = false;
        for (int v : G[j]) {
          if (v == cx || v == cy) {
            if (!flag) { nodes.push_back(cx); flag = true; }
          } else {
            nodes.push_back(v < cy ? v : v - 1);
          }
        }
        T.push_back(std::move(nodes));
      }
    }
    // redundant edges (AlignGraph.h:656-698): every test reads the old graph
    // and sets, and every edit is a removal, so they commute
    const uint64_t* Ax = anc.row(cx);
    const uint64_t* Ay = anc.row(cy);
    const uint64_t* Dx = desc.row(cx);
    const uint64_t* Dy = desc.row(cy);
    auto bit = [](const uint64_t* x, int j) { return (x[j >> 6] >> (j & 63)) & 1; };
    std::vector<std::pair<int, int>> rm;   // (new list index, value to remove)
    for_bits(Ax, n, [&](int a) {
      for (int d : G[a])
        if (bit(Dy, d)) rm.push_back({U(a), U(d)});
      if (has(G[a], cy) && !has(G[a], cx)) rm.push_back({U(a), cx});
    });
    for_bits(Ay, n, [&](int a) {
      for (int d : G[a])
        if (bit(Dx, d)) rm.push_back({U(a), U(d)});
      if (has(G[a], cx) && !has(G[a], cy)) rm.push_back({U(a), cx});
    });
    for (int j = 0; j < n; j++) {   // parents of cx / cy (GiveParent, ascending)
      if (has(G[j], cx) && bit(Ay, j) && !has(G[j], cy)) rm.push_back({U(j), cx});
      if (has(G[j], cy) && bit(Ax, j) && !has(G[j], cx)) rm.push_back({U(j), cx});
    }
    for (int c : G[cx])
      if (bit(Dy, c) && !has(G[cy], c)) rm.push_back({cx, U(c)});
    for (int c : G[cy])
      if (bit(Dx, c) && !has(G[cx], c)) rm.push_back({cx, U(c)});
    for (const auto& [li, v] : rm) remove_all(T[li], v);
    // sets (AlignGraph.h:709-751)
    std::vector<uint64_t> A(Ax, Ax + anc.words), D(Dx, Dx + desc.words);
    for (int k = 0; k < anc.words; k++) A[k] |= Ay[k];
    for (int k = 0; k < desc.words; k++) D[k] |= Dy[k];
    BitRows::drop_bit(A.data(), anc.words, cy);
    BitRows::drop_bit(D.data(), desc.words, cy);
    anc.erase_row(cy, n);
    desc.erase_row(cy, n);
    for (int j = 0; j < n - 1; j++) {
      if (j == cx) {
        memcpy(anc.row(j), A.data(), sizeof(uint64_t) * anc.words);
        memcpy(desc.row(j), D.data(), sizeof(uint64_t) * desc.words);
      } else {
        BitRows::drop_bit(anc.row(j), anc.words, cy);
        BitRows::drop_bit(desc.row(j), desc.words, cy);
      }
    }
    G.swap(T);
    // residues of cy now sit in cx; ids above cy move down one index
    const int idy = id_of[cy], idx = id_of[cx];
    for (const auto& [s, r] : members[idy]) {
      present[s][r] = idx;
      members[idx].push_back({s, r});
      seqbits[idx][s >> 6] |= 1ull << (s & 63);
    }
    members[idy].clear();
    id_of.erase(id_of.begin() + cy);
    for (int j = cy; j < n - 1; j++) idx_of[id_of[j]] = j;
    close_sets(cx, A, D, n - 1);
    return true;
  }
};

}  // namespace

Profile graph_alignment(const std::vector<Row>& seqs, const SparseSet& sp) {
  const int n = (int)seqs.size();
  // ComputeGraph (CPNP/MSA.cpp:1791-1838): every entry of every pair, pair
  // order, rows ascending, entries in row order: (a, k - 1, b, col - 1), p
  const int64_t P = (int64_t)n * (n - 1) / 2;
  const int64_t total = P ? sp.ent_off[P] : 0;
  std::vector<int32_t> ea(total), ek(total), eb(total), ec(total);
  std::vector<float> prob(total);
  {
    int64_t e = 0;
    for (int a = 0; a < n; a++)
      for (int b = a + 1; b < n; b++) {
        const int64_t p = sp.pair(a, b);
        const int32_t* rp = sp.row_ptr.data() + sp.rp_off[p];
        const int64_t e0 = sp.ent_off[p];
        for (int k = 1; k <= sp.lens[a]; k++)
          for (int32_t h = rp[k]; h < rp[k + 1]; h++, e++) {
            ea[e] = a;
            ek[e] = k - 1;
            eb[e] = b;
            ec[e] = sp.cols[e0 + h] - 1;
            prob[e] = sp.vals[e0 + h];
          }
      }
  }
  // AlignGraph::AlignGraph (AlignGraph.h:894-1089)
  std::vector<int> ind(total);
  for (int64_t i = 0; i < total; i++) ind[i] = (int)i;
  quick_sort(prob, ind);
  Graph g;
  g.nseq = n;
  for (const Row& r : seqs) g.maxlen = std::max(g.maxlen, r.length());
  g.present.assign(n, std::vector<int>(g.maxlen, -1));
  g.placed.resize(n);
  for (int64_t i = 0; i < total; i++) {
    const int e = ind[total - 1 - i];
    int xs = ea[e], xr = ek[e], ys = eb[e], yr = ec[e];
    int cx = g.node_at(xs, xr), cy = g.node_at(ys, yr);
    const bool fx = cx >= 0, fy = cy >= 0;
    if (!fx && !fy) {
      g.add_node(xs, xr, ys, yr);
    } else if (fx != fy) {
      if (fy) {   // x: the residue already in the graph
        std::swap(xs, ys);
        std::swap(xr, yr);
        std::swap(cx, cy);
      }
      if (!g.node_has_seq(cx, ys)) g.extend(ys, yr, cx);
    } else if (cx != cy) {
      if (!g.node_has_seq(cx, ys) && !g.node_has_seq(cy, xs)) {
        if (cx > cy) std::swap(cx, cy);
        g.merge(cx, cy);
      }
    }
  }
  // Graph2Align (AlignGraph.h:1096-1152): roots in index order, each put at
  // the front of the path, then a depth-first walk that puts every newly
  // reached child right after its parent
  const int nn = (int)g.G.size();
  std::vector<int> indeg(nn, 0);
  for (int i = 0; i < nn; i++)
    for (int c : g.G[i]) indeg[c]++;
  std::vector<int> next(nn, -1);
  int head = -1;
  std::vector<char> marked(nn, 0);
  std::vector<std::pair<int, int>> stack;   // (node, next child position)
  for (int r = 0; r < nn; r++) {
    if (indeg[r]) continue;
    next[r] = head;   // AddtoPath(Path, -1, root): front (or the only element)
    head = r;
    stack.push_back({r, 0});
    while (!stack.empty()) {
      auto& [u, k] = stack.back();
      if (k >= (int)g.G[u].size()) {
        stack.pop_back();
        continue;
      }
      const int c = g.G[u][k++];
      if (marked[c]) continue;
      marked[c] = 1;
      next[c] = next[u];   // AddtoPath(Path, u, c): right after u
      next[u] = c;
      stack.push_back({c, 0});   // (u, k) are not used after this: the push may move them
    }
  }
  std::vector<int> path, pos(nn, -1);
  for (int v = head; v >= 0; v = next[v]) {
    pos[v] = (int)path.size();
    path.push_back(v);
  }
  // single-residue columns after each path node, or at the very start
  std::vector<std::vector<std::pair<int, int>>> src(path.size());
  std::vector<std::pair<int, int>> zero;
  int nsingle = 0;
  for (int s = 0; s < n; s++)
    for (int r = 0; r < seqs[s].length(); r++) {
      if (g.present[s][r] >= 0) continue;
      nsingle++;
      int ct = r - 1;
      while (ct >= 0 && g.present[s][ct] < 0) ct--;
      if (ct >= 0) src[pos[g.node_at(s, ct)]].push_back({s, r});
      else zero.push_back({s, r});
    }
  // Path2Align (AlignGraph.h:808-874); cols[node] in (sequence, residue) order
  std::vector<std::vector<int>> col_res(nn);   // per node: residue of each sequence or -1
  Profile out(n);
  const size_t width = path.size() + nsingle;
  for (int s = 0; s < n; s++) {
    out[s].header = seqs[s].header;
    out[s].label = seqs[s].label;
    out[s].sort_label = seqs[s].sort_label;
    out[s].data.reserve(width + 1);
    out[s].data = "@";
  }
  auto single = [&](int s, int r) {
    for (int k = 0; k < n; k++) out[k].data += k == s ? seqs[s].data[r + 1] : '-';
  };
  for (const auto& [s, r] : zero) single(s, r);
  std::vector<int> res_of(n);
  for (size_t i = 0; i < path.size(); i++) {
    std::fill(res_of.begin(), res_of.end(), -1);
    for (const auto& [s, r] : g.members[g.id_of[path[i]]]) res_of[s] = r;
    for (int s = 0; s < n; s++) out[s].data += res_of[s] >= 0 ? seqs[s].data[res_of[s] + 1] : '-';
    for (const auto& [s, r] : src[i]) single(s, r);
  }
  return out;
}

// ---------------------------------------------------------------- refinement
// MSA::FindSimilar (CPNP/MSA.cpp:1986-2082): for each sequence, a two-means
// split of its row of the npdoAlign distances (score / #B: larger = closer)
static std::vector<std::set<int>> find_similar(std::vector<std::vector<float>> d) {
  const int n = (int)d.size();
  for (int i = 0; i < n; i++) d[i][i] = 1;
  std::vector<std::set<int>> sim;
  for (int i = 0; i < n; i++) {
    std::set<int> c1, c2;
    float min_d = 1, max_d = 0;
    int ii_min = 0, ii_max = 0;
    for (int j = 0; j < n; j++) {
      if (d[i][j] <= min_d) { ii_min = j; min_d = d[i][j]; }
      if (d[i][j] >= max_d) { ii_max = j; max_d = d[i][j]; }
    }
    c1.insert(ii_max);
    c2.insert(ii_min);
    for (int j = 0; j < n; j++)
      if (j != ii_min && j != ii_max) {
        if (std::fabs(d[j][i] - max_d) < std::fabs(d[j][i] - min_d)) c1.insert(j);
        else c2.insert(j);
      }
    if (!c1.count(i)) {
      c2.erase(i);
      c1.insert(i);
    }
    bool changed = true;
    for (int it = 0; it < 100 && changed; it++) {
      changed = false;
      std::vector<int> ch(n, 0);
      float m1 = 0, m2 = 0;
      for (int k : c1) m1 += d[i][k];
      for (int k : c2) m2 += d[i][k];
      m1 /= (float)c1.size();
      m2 /= (float)c2.size();
      for (int j = 0; j < n; j++) {
        if (j == i) continue;
        if (c1.count(j)) {
          if (std::fabs(d[j][i] - m1) > std::fabs(d[j][i] - m2)) { ch[j] = 1; changed = true; }
        } else {
          if (std::fabs(d[j][i] - m2) > std::fabs(d[j][i] - m1)) { ch[j] = -1; changed = true; }
        }
      }
      if (changed)
        for (int j = 0; j < n; j++) {
          if (ch[j] == 1) { c1.erase(j); c2.insert(j); }
          else if (ch[j] == -1) { c2.erase(j); c1.insert(j); }
        }
    }
    sim.push_back(std::move(c1));
  }
  return sim;
}

// AlignAlignments(..., nflag = false) (CPNP/MSA.cpp:1410-1471): unweighted
// profile posterior, MEA, merge, SortByLabel unless -a
static Profile align_profiles(const Profile& a, const Profile& b, const SparseSet& sp, const Options& opt,
                              float* score) {
  std::string path;
  if (!device_mea(a, b, nullptr, opt.cutoff, nullptr, nullptr, path, score)) {
    const float* post = profile_posterior(a, b, sp, nullptr, opt.cutoff);
    path = mea_path(a[0].length(), b[0].length(), post, score);
  }
  return merge(a, b, path, !opt.align_order);
}

static uint32_t refinement_seed() {   // srand(time(0)) (CPNP/MSA.cpp:1896)
  static const char* fixed = getenv("MLP_SRAND_TIME");   // test hook: a fixed clock
  return fixed ? (uint32_t)strtoul(fixed, nullptr, 10) : (uint32_t)time(nullptr);
}

// MSA::DoRefinement (CPNP/MSA.cpp:1852-1978)
Profile np_refinement(Profile aln, const SparseSet& sp, const std::vector<std::vector<float>>& dist,
                      const Options& opt) {
  const int n = (int)aln.size();
  int reps = n > 150 ? 0 : opt.refinement;
  const std::vector<std::set<int>> sim = find_similar(dist);
  int cnt = 0, ineffective = 0;
  float oscore = 0, nscore = 0;
  while (cnt < reps) {
    libc_srand(refinement_seed());
    std::vector<int> list(n), order;
    for (int i = 0; i < n; i++) list[i] = i;
    while (!list.empty()) {   // a random permutation by rand() % remaining
      const int k = libc_rand_next() % (int)list.size();
      order.push_back(list[k]);
      list.erase(list.begin() + k);
    }
    for (int i = 0; i < n; i++) {
      const int si = order[i];
      const std::set<int>& one = sim[si];
      std::set<int> two;
      for (int j = 0; j < n; j++)
        if (!one.count(j)) two.insert(j);
      cnt++;
      if (one.empty() || two.empty()) continue;
      Profile g1 = project(aln, one);
      const Profile g2 = project(aln, two);
      int at = 0;   // position of si in S_x
      for (int k : one) {
        if (k == si) break;
        at++;
      }
      float oscore2 = 0, nscore2 = 0;
      if (g1.size() > 1) {   // update S_x by aligning x with S_x - x
        std::set<int> only{at}, rest;
        for (int k = 0; k < (int)g1.size(); k++)
          if (k != at) rest.insert(k);
        const Profile x = project(g1, only), others = project(g1, rest);
        g1 = align_profiles(x, others, sp, opt, &nscore2);
        if (nscore2 > oscore2) oscore2 = nscore2;
        else ineffective++;
        cnt++;
      }
      aln = align_profiles(g1, g2, sp, opt, &nscore);
      if (nscore < oscore && reps < 8 * n && ineffective < 4 * n) {
        oscore = nscore;
        reps += n;
      }
    }
  }
  return aln;
}

}  // namespace cpnp
