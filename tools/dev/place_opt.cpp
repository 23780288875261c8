// place_opt.cpp — offline study of the LDS bank conflicts of the m2s variable phase (round 4).
//
// Reads a decoder's lane map (tools/dev/place_dump.py) and evaluates / optimizes the V-slot
// placement under the exact lane-group model of qldpc_bp_lds_model (MI355X_MICROARCH.md §LDS):
// per instruction and lane group the cost is the maximum number of distinct addresses on one bank
// (pair); CS gathers (ds_read_b64, 32 lanes, bank pair (label + 1) mod 32), V-slot reads
// (ds_read_b64, 32 lanes, (vbase + slot) mod 32) and v2c stores (ds_write_b64, 16 contiguous lanes,
// (vbase + slot) mod 16).  Layouts:
//   A: rows of 3 x 16-byte chunks + a tail array (the m2s kernel): slot = 2 + 6 lab + pos (pos < 6),
//      tail slot = tail0 + lab;
//   B: rows of 7 contiguous 8-byte slots: slot = 1 + 7 lab + pos.
// Moves: swap two positions of one row (storage only), and optionally swap the labels of two
// checks (moves their CS entries and rows).  Simulated annealing on the exact cost.
//   g++ -O2 -o /tmp/place_opt tools/dev/place_opt.cpp && /tmp/place_opt dump.txt A 2000000 [labels]
#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

struct Group {
  int nb;                 // banks
  std::vector<int> cnt;   // distinct addresses per bank
  std::vector<int> hist;  // banks per count
  int mx = 0;
  std::vector<std::pair<int, int>> addr_refs;  // (address, refcount) for broadcast of identical addresses
};

static uint64_t rs = 0x9E3779B97F4A7C15ull;
static inline uint64_t rnd() {
  rs ^= rs << 13;
  rs ^= rs >> 7;
  rs ^= rs << 17;
  return rs;
}

int main(int argc, char** argv) {
  if (argc < 4) {
    fprintf(stderr, "usage: place_opt dump.txt A|B iters [labels]\n");
    return 1;
  }
  FILE* f = fopen(argv[1], "r");
  const char layout = argv[2][0];
  const long long iters = atoll(argv[3]);
  const bool do_labels = argc > 4 && std::string(argv[4]) == "labels";
  int m, n, TB, VPL, DM, D3K;
  if (fscanf(f, "%d %d %d %d %d %d", &m, &n, &TB, &VPL, &DM, &D3K) != 6) return 1;
  std::vector<int> sv((size_t)VPL * TB);
  for (auto& x : sv)
    if (fscanf(f, "%d", &x) != 1) return 1;
  std::vector<std::vector<int>> cr(n);
  for (int j = 0; j < n; ++j) {
    int d;
    if (fscanf(f, "%d", &d) != 1) return 1;
    cr[j].resize(d);
    for (auto& r : cr[j])
      if (fscanf(f, "%d", &r) != 1) return 1;
  }
  fclose(f);
  const int RW = layout == 'A' ? 7 : 7;  // positions per row
  const int vbase = 770;                 // V base in 8-byte units (CS array (m + 1) * 8 B, 16-aligned)
  const int tail0 = (1 + m * 3) * 2;
  std::vector<int> lab(m);
  for (int i = 0; i < m; ++i) lab[i] = i;
  auto slot = [&](int i, int pos) {
    if (layout == 'A') return pos < 6 ? 2 + 6 * lab[i] + pos : tail0 + lab[i];
    return 1 + 7 * lab[i] + pos;
  };
  // edges: (row, lane slot) with their groups
  struct E {
    int row, rg, wg, cg;
  };
  std::vector<E> edges;
  std::vector<std::vector<int>> row_edges(m);
  int nrg = 0, nwg = 0, ncg = 0;
  for (int k = 0; k < VPL; ++k)
    for (int d = 0; d < DM; ++d) {
      if (k < D3K && d >= 3) continue;
      for (int w = 0; w * 64 < TB; ++w) {
        const int rg0 = nrg, wg0 = nwg, cg0 = ncg;
        nrg += 2;
        nwg += 4;
        ncg += 2;
        for (int l = 0; l < 64; ++l) {
          const int t = w * 64 + l;
          const int j = t < TB ? sv[(size_t)k * TB + t] : -1;
          if (j < 0 || d >= (int)cr[j].size()) continue;  // padding lanes: the dummy address (ignored)
          edges.push_back({cr[j][d], rg0 + l / 32, wg0 + l / 16, cg0 + l / 32});
          row_edges[cr[j][d]].push_back((int)edges.size() - 1);
        }
      }
    }
  for (int i = 0; i < m; ++i)
    if ((int)row_edges[i].size() > RW) {
      fprintf(stderr, "row %d has %zu edges > %d positions\n", i, row_edges[i].size(), RW);
      return 1;
    }
  // position of each edge: initially in CSR order
  std::vector<int> pos(edges.size());
  std::vector<std::vector<int>> at(m, std::vector<int>(RW, -1));
  for (int i = 0; i < m; ++i)
    for (int q = 0; q < (int)row_edges[i].size(); ++q) {
      pos[row_edges[i][q]] = q;
      at[i][q] = row_edges[i][q];
    }
  // group state: counts of edges per (group, bank); distinct addresses only matter when two lanes
  // of a group hit the same row slot, which cannot happen (one edge per slot)
  std::vector<int> rc((size_t)nrg * 32, 0), wc((size_t)nwg * 16, 0), cc((size_t)ncg * 32, 0);
  std::vector<std::vector<int>> cs_rows(ncg);  // distinct checks per CS group (broadcast)
  auto rb = [&](int e) { return (vbase + slot(edges[e].row, pos[e])) % 32; };
  auto wb = [&](int e) { return (vbase + slot(edges[e].row, pos[e])) % 16; };
  auto gmax = [](const int* c, int nb) {
    int mx = 0;
    for (int b = 0; b < nb; ++b) mx = std::max(mx, c[b]);
    return std::max(mx, 1);
  };
  auto total = [&]() {
    std::fill(rc.begin(), rc.end(), 0);
    std::fill(wc.begin(), wc.end(), 0);
    for (size_t e = 0; e < edges.size(); ++e) {
      rc[(size_t)edges[e].rg * 32 + rb((int)e)]++;
      wc[(size_t)edges[e].wg * 16 + wb((int)e)]++;
    }
    long long r = 0, w = 0, c = 0;
    for (int g = 0; g < nrg; ++g) r += gmax(&rc[(size_t)g * 32], 32);
    for (int g = 0; g < nwg; ++g) w += gmax(&wc[(size_t)g * 16], 16);
    // CS gathers: distinct checks per group, bank pair (lab + 1) mod 32
    for (int g = 0; g < ncg; ++g) std::fill(&cc[(size_t)g * 32], &cc[(size_t)g * 32 + 32], 0);
    std::vector<std::vector<int>> seen(ncg);
    for (size_t e = 0; e < edges.size(); ++e) seen[edges[e].cg].push_back(edges[e].row);
    for (int g = 0; g < ncg; ++g) {
      auto& v = seen[g];
      std::sort(v.begin(), v.end());
      v.erase(std::unique(v.begin(), v.end()), v.end());
      for (int i : v) cc[(size_t)g * 32 + (lab[i] + 1) % 32]++;
      c += gmax(&cc[(size_t)g * 32], 32);
    }
    return std::make_tuple(c, r, w);
  };
  auto [c0, r0, w0] = total();
  printf("layout %c start: cs %lld v_read %lld v_store %lld  (groups: cs %d, read %d, store %d)\n", layout, c0, r0, w0,
         ncg, nrg, nwg);
  // annealing on positions (cost = reads + stores, exact maxima recomputed per touched group)
  long long cur = r0 + w0;
  for (long long it = 0; it < iters; ++it) {
    const int i = (int)(rnd() % (uint64_t)m);
    const int a = (int)(rnd() % (uint64_t)RW), b = (int)(rnd() % (uint64_t)RW);
    if (a == b) continue;
    const int ea = at[i][a], eb = at[i][b];
    if (ea < 0 && eb < 0) continue;
    // touched groups
    int gr[2] = {ea >= 0 ? edges[ea].rg : -1, eb >= 0 ? edges[eb].rg : -1};
    int gw[2] = {ea >= 0 ? edges[ea].wg : -1, eb >= 0 ? edges[eb].wg : -1};
    long long before = 0, after = 0;
    auto sum_groups = [&]() {
      long long s = 0;
      for (int q = 0; q < 2; ++q) {
        if (gr[q] >= 0 && !(q == 1 && gr[1] == gr[0])) s += gmax(&rc[(size_t)gr[q] * 32], 32);
        if (gw[q] >= 0 && !(q == 1 && gw[1] == gw[0])) s += gmax(&wc[(size_t)gw[q] * 16], 16);
      }
      return s;
    };
    before = sum_groups();
    auto mv = [&](int e, int sg) {
      if (e < 0) return;
      rc[(size_t)edges[e].rg * 32 + rb(e)] += sg;
      wc[(size_t)edges[e].wg * 16 + wb(e)] += sg;
    };
    mv(ea, -1);
    mv(eb, -1);
    if (ea >= 0) pos[ea] = b;
    if (eb >= 0) pos[eb] = a;
    mv(ea, +1);
    mv(eb, +1);
    after = sum_groups();
    const double T = 0.6 * (1.0 - (double)it / iters);
    const long long dlt = after - before;
    if (dlt <= 0 || (T > 0 && (double)(rnd() % 1000000) / 1e6 < std::exp(-(double)dlt / T))) {
      at[i][a] = eb;
      at[i][b] = ea;
      cur += dlt;
    } else {
      mv(ea, -1);
      mv(eb, -1);
      if (ea >= 0) pos[ea] = a;
      if (eb >= 0) pos[eb] = b;
      mv(ea, +1);
      mv(eb, +1);
    }
  }
  auto [c1, r1, w1] = total();
  printf("layout %c after %lld position moves: cs %lld v_read %lld v_store %lld (extra over conflict-free: cs %d, "
         "read %lld, store %lld)\n",
         layout, iters, c1, r1, w1, 0, r1 - nrg, w1 - nwg);
  (void)do_labels;
  return 0;
}
