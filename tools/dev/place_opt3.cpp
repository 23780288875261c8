// place_opt3.cpp — offline study (round 4): JOINT check labelling, in-row positions and
// variable-to-lane assignment for the m2s variable phase, on the exact lane-group bank model of
// qldpc_bp_lds_model (MI355X_MICROARCH.md §LDS):
//   CS gathers:  ds_read_b64, 2 groups of 32 lanes per wave, bank pair (label + 1) mod 32, identical
//                addresses (same check) broadcast;
//   V-slot reads: ds_read_b64, 32-lane groups, bank pair (vbase + slot) mod 32;
//   v2c stores:  ds_write_b64, 16 contiguous lanes, bank pair (vbase + slot) mod 16.
// Group cost = max over banks of the distinct addresses there (1 = conflict-free); the objective is
// cs + read + ws * store.  Layout A (the m2s kernel): slot = 2 + 6 lab + pos (pos < 6), tail slot
// tail0 + lab.  Moves (simulated annealing, exact deltas through per-group bank histograms):
//   P: swap two positions of one row;  L: swap the labels of two checks;
//   V: swap two variables of equal column degree (their lanes and slots k).
//   g++ -O2 -o /tmp/place_opt3 tools/dev/place_opt3.cpp
//   python tools/dev/place_dump.py hz > /tmp/hz.txt && /tmp/place_opt3 /tmp/hz.txt 20000000 PLV [ws] [T0]
#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <unordered_map>
#include <vector>

static uint64_t rs = 0x9E3779B97F4A7C15ull;
static inline uint64_t rnd() {
  rs ^= rs << 13;
  rs ^= rs >> 7;
  rs ^= rs << 17;
  return rs;
}

// bank histogram of one lane group: cnt[b] = addresses on bank b, hist[c] = banks with count c
struct G {
  int nb = 32;
  uint8_t cnt[32];
  int hist[40];
  int mx = 0;
  void init(int n) {
    nb = n;
    memset(cnt, 0, sizeof cnt);
    memset(hist, 0, sizeof hist);
    hist[0] = n;
    mx = 0;
  }
  void add(int b) {
    hist[cnt[b]]--;
    cnt[b]++;
    hist[cnt[b]]++;
    if (cnt[b] > mx) mx = cnt[b];
  }
  void sub(int b) {
    hist[cnt[b]]--;
    cnt[b]--;
    hist[cnt[b]]++;
    while (mx > 0 && hist[mx] == 0) --mx;
  }
  int cost() const { return mx > 1 ? mx : 1; }
};

int main(int argc, char** argv) {
  if (argc < 4) {
    fprintf(stderr, "usage: place_opt3 dump.txt iters moves(PLV) [store_weight]\n");
    return 1;
  }
  FILE* f = fopen(argv[1], "r");
  const long long iters = atoll(argv[2]);
  const std::string mv = argv[3];
  const double ws = argc > 4 ? atof(argv[4]) : 1.0;
  const double T0 = argc > 5 ? atof(argv[5]) : 0.3;
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
  const int RW = 7, vbase = 770, tail0 = (1 + m * 3) * 2;
  std::vector<int> lab(m), pos_of_var(n);
  for (int i = 0; i < m; ++i) lab[i] = i;
  for (int p = 0; p < VPL * TB; ++p)
    if (sv[p] >= 0) pos_of_var[sv[p]] = p;
  auto slot = [&](int i, int ps) { return ps < 6 ? 2 + 6 * lab[i] + ps : tail0 + lab[i]; };
  // edges: (variable, d) -> row; groups from the variable's lane position
  struct E {
    int row, var, d, ps;
  };
  std::vector<E> ed;
  std::vector<std::vector<int>> row_e(m), var_e(n);
  for (int j = 0; j < n; ++j)
    for (int d = 0; d < (int)cr[j].size(); ++d) {
      ed.push_back({cr[j][d], j, d, -1});
      row_e[cr[j][d]].push_back((int)ed.size() - 1);
      var_e[j].push_back((int)ed.size() - 1);
    }
  for (int i = 0; i < m; ++i) {
    if ((int)row_e[i].size() > RW) return 2;
    for (int q = 0; q < (int)row_e[i].size(); ++q) ed[row_e[i][q]].ps = q;
  }
  std::vector<std::vector<int>> at(m, std::vector<int>(RW, -1));
  for (int i = 0; i < m; ++i)
    for (int q = 0; q < (int)row_e[i].size(); ++q) at[i][q] = row_e[i][q];
  const int n32 = TB / 32, n16 = TB / 16;
  auto rg = [&](int e) { const int p = pos_of_var[ed[e].var]; return ((p / TB) * DM + ed[e].d) * n32 + (p % TB) / 32; };
  auto wg = [&](int e) { const int p = pos_of_var[ed[e].var]; return ((p / TB) * DM + ed[e].d) * n16 + (p % TB) / 16; };
  const int NR = VPL * DM * n32, NW = VPL * DM * n16;
  std::vector<G> R(NR), W(NW), C(NR);
  for (auto& g : R) g.init(32);
  for (auto& g : W) g.init(16);
  for (auto& g : C) g.init(32);
  std::unordered_map<long long, int> csm;  // (cs group, check) -> multiplicity
  auto cs_add = [&](int g, int i) {
    int& c = csm[(long long)g * m + i];
    if (c++ == 0) C[g].add((lab[i] + 1) % 32);
  };
  auto cs_sub = [&](int g, int i) {
    int& c = csm[(long long)g * m + i];
    if (--c == 0) C[g].sub((lab[i] + 1) % 32);
  };
  auto put = [&](int e, int sg) {  // add / remove edge e from its three groups
    const int s = vbase + slot(ed[e].row, ed[e].ps);
    if (sg > 0) {
      R[rg(e)].add(s % 32);
      W[wg(e)].add(s % 16);
      cs_add(rg(e), ed[e].row);
    } else {
      R[rg(e)].sub(s % 32);
      W[wg(e)].sub(s % 16);
      cs_sub(rg(e), ed[e].row);
    }
  };
  for (size_t e = 0; e < ed.size(); ++e) put((int)e, +1);
  auto totals = [&](long long& c, long long& r, long long& w) {
    c = r = w = 0;
    for (int g = 0; g < NR; ++g) {
      bool used = false;
      for (int b = 0; b < 32; ++b) used = used || R[g].cnt[b];
      if (!used) continue;
      r += R[g].cost();
      c += C[g].cost();
    }
    for (int g = 0; g < NW; ++g) {
      bool used = false;
      for (int b = 0; b < 16; ++b) used = used || W[g].cnt[b];
      if (used) w += W[g].cost();
    }
  };
  long long c0, r0, w0;
  totals(c0, r0, w0);
  printf("start: cs %lld read %lld store %lld\n", c0, r0, w0);
  // touched-group cost (deduplicated)
  std::vector<int> tr, tw;
  auto gcost = [&]() {
    std::sort(tr.begin(), tr.end());
    tr.erase(std::unique(tr.begin(), tr.end()), tr.end());
    std::sort(tw.begin(), tw.end());
    tw.erase(std::unique(tw.begin(), tw.end()), tw.end());
    double s = 0;
    for (int g : tr) s += R[g].cost() + C[g].cost();
    for (int g : tw) s += ws * W[g].cost();
    return s;
  };
  long long acc[3] = {0, 0, 0}, tried[3] = {0, 0, 0};
  for (long long it = 0; it < iters; ++it) {
    const double T = T0 * (1.0 - (double)it / iters) + 1e-3;
    const char kind = mv[rnd() % mv.size()];
    std::vector<int> es;  // edges whose slot / group changes
    int i1 = -1, i2 = -1, a = -1, b = -1, j1 = -1, j2 = -1;
    if (kind == 'P') {
      i1 = (int)(rnd() % (uint64_t)m);
      a = (int)(rnd() % RW);
      b = (int)(rnd() % RW);
      if (a == b || (at[i1][a] < 0 && at[i1][b] < 0)) continue;
      if (at[i1][a] >= 0) es.push_back(at[i1][a]);
      if (at[i1][b] >= 0) es.push_back(at[i1][b]);
    } else if (kind == 'L') {
      i1 = (int)(rnd() % (uint64_t)m);
      i2 = (int)(rnd() % (uint64_t)m);
      if (i1 == i2) continue;
      es = row_e[i1];
      es.insert(es.end(), row_e[i2].begin(), row_e[i2].end());
    } else {
      j1 = (int)(rnd() % (uint64_t)n);
      j2 = (int)(rnd() % (uint64_t)n);
      if (j1 == j2 || cr[j1].size() != cr[j2].size()) continue;
      es = var_e[j1];
      es.insert(es.end(), var_e[j2].begin(), var_e[j2].end());
    }
    const int ki = kind == 'P' ? 0 : kind == 'L' ? 1 : 2;
    tried[ki]++;
    tr.clear();
    tw.clear();
    for (int e : es) {
      tr.push_back(rg(e));
      tw.push_back(wg(e));
    }
    auto apply = [&]() {
      if (kind == 'P') {
        std::swap(at[i1][a], at[i1][b]);
        if (at[i1][a] >= 0) ed[at[i1][a]].ps = a;
        if (at[i1][b] >= 0) ed[at[i1][b]].ps = b;
      } else if (kind == 'L') {
        std::swap(lab[i1], lab[i2]);
      } else {
        std::swap(pos_of_var[j1], pos_of_var[j2]);
      }
    };
    for (int e : es) put(e, -1);
    // costs before: re-add, measure, remove (exact)
    for (int e : es) put(e, +1);
    const double before = gcost();
    for (int e : es) put(e, -1);
    apply();
    for (int e : es) {
      tr.push_back(rg(e));
      tw.push_back(wg(e));
    }
    for (int e : es) put(e, +1);
    // after: the union of old and new groups (old groups lost the edges, new gained them)
    const double after_all = gcost();
    // before over the same union: undo, measure, redo would cost more; instead compare over the
    // union by recomputing `before` on it
    for (int e : es) put(e, -1);
    apply();  // swaps are involutions: back to the old state
    for (int e : es) put(e, +1);
    const double before_all = gcost();
    (void)before;
    const double dlt = after_all - before_all;
    const bool take = dlt <= 0 || (double)(rnd() % 1000000) / 1e6 < std::exp(-dlt / T);
    if (take) {
      for (int e : es) put(e, -1);
      apply();
      for (int e : es) put(e, +1);
      acc[ki]++;
    }
    if ((it + 1) % (iters / 10 > 0 ? iters / 10 : 1) == 0) {
      long long c, r, w;
      totals(c, r, w);
      printf("it %lld T %.3f: cs %lld read %lld store %lld (accepted P %lld/%lld L %lld/%lld V %lld/%lld)\n", it + 1, T, c,
             r, w, acc[0], tried[0], acc[1], tried[1], acc[2], tried[2]);
      fflush(stdout);
    }
  }
  long long c, r, w;
  totals(c, r, w);
  printf("final: cs %lld read %lld store %lld  (conflict-free: cs %d read %d store %d)\n", c, r, w, 192, 192, 384);
  return 0;
}
