// place_opt4.cpp — offline study (round 4): "layout C" for the m2s variable phase: every row is 8
// aligned 8-byte slots (slot = 8 lab + pos, pos < 8) holding its 7 edges' V slots AND its CS word at
// a per-row position cs(lab), i.e. the same 52 KiB image as the current 3 chunks + tail + CS array.
// Aligned rows make the bank of slot (lab, pos) = (c0 + 8 (lab mod 4) + pos) mod 32 for 32-lane
// reads, (c0 + 8 (lab mod 2) + pos) mod 16 for 16-lane stores: with the labels' classes balanced per
// lane group, conflict-free reads / stores / CS gathers are an edge colouring.  Annealing over
// label swaps (L), in-row position swaps including the CS position (P) on the exact lane-group
// model of qldpc_bp_lds_model.
//   g++ -O2 -o /tmp/place_opt4 tools/dev/place_opt4.cpp && /tmp/place_opt4 /tmp/hz.txt 20000000 PL [T0]
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
struct G {
  uint8_t cnt[32];
  int hist[64];
  int mx = 0;
  void init() {
    memset(cnt, 0, sizeof cnt);
    memset(hist, 0, sizeof hist);
    hist[0] = 32;
    mx = 0;
  }
  void add(int b) { hist[cnt[b]]--; hist[++cnt[b]]++; if (cnt[b] > mx) mx = cnt[b]; }
  void sub(int b) { hist[cnt[b]]--; hist[--cnt[b]]++; while (mx > 0 && hist[mx] == 0) --mx; }
  int cost() const { return mx > 1 ? mx : 1; }
};

int main(int argc, char** argv) {
  FILE* f = fopen(argv[1], "r");
  const long long iters = atoll(argv[2]);
  const std::string mv = argv[3];
  const double T0 = argc > 4 ? atof(argv[4]) : 0.05;
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
  const int c0 = 0;  // V base in 8-byte units mod 32 (aligned)
  std::vector<int> lab(m), pos_of_var(n);
  for (int i = 0; i < m; ++i) lab[i] = i;
  for (int p = 0; p < VPL * TB; ++p)
    if (sv[p] >= 0) pos_of_var[sv[p]] = p;
  struct E {
    int row, var, d, ps;
  };
  std::vector<E> ed;
  std::vector<std::vector<int>> row_e(m);
  for (int j = 0; j < n; ++j)
    for (int d = 0; d < (int)cr[j].size(); ++d) {
      ed.push_back({cr[j][d], j, d, -1});
      row_e[cr[j][d]].push_back((int)ed.size() - 1);
    }
  // at[i][pos] = edge, or -2 = the CS word, -1 = free
  std::vector<std::vector<int>> at(m, std::vector<int>(8, -1));
  for (int i = 0; i < m; ++i) {
    for (int q = 0; q < (int)row_e[i].size(); ++q) {
      at[i][q] = row_e[i][q];
      ed[row_e[i][q]].ps = q;
    }
    at[i][7] = -2;
  }
  auto cspos = [&](int i) {
    for (int q = 0; q < 8; ++q)
      if (at[i][q] == -2) return q;
    return -1;
  };
  const int n32 = TB / 32, n16 = TB / 16;
  auto rg = [&](int e) { const int p = pos_of_var[ed[e].var]; return ((p / TB) * DM + ed[e].d) * n32 + (p % TB) / 32; };
  auto wg = [&](int e) { const int p = pos_of_var[ed[e].var]; return ((p / TB) * DM + ed[e].d) * n16 + (p % TB) / 16; };
  const int NR = VPL * DM * n32, NW = VPL * DM * n16;
  std::vector<G> R(NR), W(NW), C(NR);
  for (auto& g : R) g.init();
  for (auto& g : W) g.init();
  for (auto& g : C) g.init();
  std::unordered_map<long long, int> csm;
  auto slot = [&](int i, int q) { return c0 + 8 * lab[i] + q; };
  auto put = [&](int e, int sg) {
    const int i = ed[e].row, s = slot(i, ed[e].ps), g = rg(e);
    const int cb = slot(i, cspos(i)) % 32;
    if (sg > 0) {
      R[g].add(s % 32);
      W[wg(e)].add(s % 16);
      if (csm[(long long)g * m + i]++ == 0) C[g].add(cb);
    } else {
      R[g].sub(s % 32);
      W[wg(e)].sub(s % 16);
      if (--csm[(long long)g * m + i] == 0) C[g].sub(cb);
    }
  };
  for (size_t e = 0; e < ed.size(); ++e) put((int)e, +1);
  std::vector<char> usedR(NR, 0), usedW(NW, 0);
  for (size_t e = 0; e < ed.size(); ++e) {
    usedR[rg((int)e)] = 1;
    usedW[wg((int)e)] = 1;
  }
  auto totals = [&](long long& c, long long& r, long long& w) {
    c = r = w = 0;
    for (int g = 0; g < NR; ++g)
      if (usedR[g]) {
        r += R[g].cost();
        c += C[g].cost();
      }
    for (int g = 0; g < NW; ++g)
      if (usedW[g]) w += W[g].cost();
  };
  long long c, r, w;
  totals(c, r, w);
  long long ng = 0, nw = 0;
  for (int g = 0; g < NR; ++g) ng += usedR[g];
  for (int g = 0; g < NW; ++g) nw += usedW[g];
  printf("groups: read/cs %lld store %lld\nstart: cs %lld read %lld store %lld\n", ng, nw, c, r, w);
  std::vector<int> tr, tw;
  auto gcost = [&]() {
    std::sort(tr.begin(), tr.end());
    tr.erase(std::unique(tr.begin(), tr.end()), tr.end());
    std::sort(tw.begin(), tw.end());
    tw.erase(std::unique(tw.begin(), tw.end()), tw.end());
    double s = 0;
    for (int g : tr) s += R[g].cost() + C[g].cost();
    for (int g : tw) s += W[g].cost();
    return s;
  };
  for (long long it = 0; it < iters; ++it) {
    const double T = T0 * (1.0 - (double)it / iters) + 1e-4;
    const char kind = mv[rnd() % mv.size()];
    int i1 = -1, i2 = -1, a = -1, b = -1;
    std::vector<int> es;
    if (kind == 'P') {
      i1 = (int)(rnd() % (uint64_t)m);
      a = (int)(rnd() % 8);
      b = (int)(rnd() % 8);
      if (a == b) continue;
      es = row_e[i1];  // (a CS move changes every CS group of the row)
    } else {
      i1 = (int)(rnd() % (uint64_t)m);
      i2 = (int)(rnd() % (uint64_t)m);
      if (i1 == i2) continue;
      es = row_e[i1];
      es.insert(es.end(), row_e[i2].begin(), row_e[i2].end());
    }
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
      } else {
        std::swap(lab[i1], lab[i2]);
      }
    };
    const double before = gcost();
    for (int e : es) put(e, -1);
    apply();
    for (int e : es) put(e, +1);
    const double dlt = gcost() - before;
    if (!(dlt <= 0 || (double)(rnd() % 1000000) / 1e6 < std::exp(-dlt / T))) {
      for (int e : es) put(e, -1);
      apply();
      for (int e : es) put(e, +1);
    }
    if ((it + 1) % (iters / 5 > 0 ? iters / 5 : 1) == 0) {
      totals(c, r, w);
      printf("it %lld: cs %lld read %lld store %lld\n", it + 1, c, r, w);
      fflush(stdout);
    }
  }
  totals(c, r, w);
  printf("final: cs %lld read %lld store %lld  (conflict-free: %lld / %lld / %lld)\n", c, r, w, ng, ng, nw);
  return 0;
}
