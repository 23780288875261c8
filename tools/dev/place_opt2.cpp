// place_opt2.cpp — as place_opt.cpp, plus lane moves: two variables of the same degree class swap
// lanes (slot k, lane t), which changes the lane groups their edges' V accesses fall in (storage
// only: the decode of a variable does not depend on its lane).  Objective: exact Σ over groups of
// the maximum bank load (reads: 32-lane groups mod 32; stores: 16-lane groups mod 16) for layout
// A (3 chunks + tail) or B (7 contiguous slots per row).  Prints the CS-gather cost too (its groups
// also move with the lanes).
//   g++ -O2 -std=c++17 -o /tmp/place_opt2 tools/dev/place_opt2.cpp
//   /tmp/place_opt2 dump.txt A|B iters lane_frac wcs
#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <vector>

static uint64_t rs = 0x9E3779B97F4A7C15ull;
static inline uint64_t rnd() {
  rs ^= rs << 13;
  rs ^= rs >> 7;
  rs ^= rs << 17;
  return rs;
}

int main(int argc, char** argv) {
  FILE* f = fopen(argv[1], "r");
  const char layout = argv[2][0];
  const long long iters = atoll(argv[3]);
  const double lane_frac = argc > 4 ? atof(argv[4]) : 0.3;
  const int wcs = argc > 5 ? atoi(argv[5]) : 1;  // weight of the CS gathers in the objective
  const int wst = argc > 6 ? atoi(argv[6]) : 1;  // weight of the v2c stores (transfer-bound up to 6 cycles)
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
  const int RW = 7, vbase = 770, tail0 = (1 + m * 3) * 2, W = TB / 64;
  auto slot = [&](int i, int p) {
    if (layout == 'A') return p < 6 ? 2 + 6 * i + p : tail0 + i;
    return 1 + 7 * i + p;
  };
  // edge e = (variable j, index d): row cr[j][d], position pos[e]
  std::vector<int> ebase(n + 1, 0);
  for (int j = 0; j < n; ++j) ebase[j + 1] = ebase[j] + (int)cr[j].size();
  const int E = ebase[n];
  std::vector<int> erow(E), pos(E, -1);
  for (int j = 0; j < n; ++j)
    for (int d = 0; d < (int)cr[j].size(); ++d) erow[ebase[j] + d] = cr[j][d];
  std::vector<std::vector<int>> at(m, std::vector<int>(RW, -1));
  for (int j = 0; j < n; ++j)
    for (int d = 0; d < (int)cr[j].size(); ++d) {
      const int i = cr[j][d], e = ebase[j] + d;
      int p = 0;
      while (at[i][p] >= 0) ++p;
      at[i][p] = e;
      pos[e] = p;
    }
  std::vector<int> lane(n);  // k * TB + t of variable j
  for (int s = 0; s < VPL * TB; ++s)
    if (sv[s] >= 0) lane[sv[s]] = s;
  auto rg = [&](int j, int d) {
    const int k = lane[j] / TB, t = lane[j] % TB;
    return ((k * DM + d) * W + t / 64) * 2 + (t % 64) / 32;
  };
  auto wg = [&](int j, int d) {
    const int k = lane[j] / TB, t = lane[j] % TB;
    return ((k * DM + d) * W + t / 64) * 4 + (t % 64) / 16;
  };
  const int NRG = VPL * DM * W * 2, NWG = VPL * DM * W * 4;
  std::vector<int> rc((size_t)NRG * 32, 0), wc((size_t)NWG * 16, 0), cc((size_t)NRG * 32, 0);
  // CS gathers: distinct rows per group (refcount per (group, row) for broadcast)
  std::vector<std::vector<std::pair<int, int>>> crow(NRG);
  auto gmax = [](const int* c, int nb) {
    int mx = 0;
    for (int b = 0; b < nb; ++b) mx = std::max(mx, c[b]);
    return mx;
  };
  auto ev_of = [&](int e) { return (int)(std::upper_bound(ebase.begin(), ebase.end(), e) - ebase.begin()) - 1; };
  std::vector<int> evar(E);
  for (int j = 0; j < n; ++j)
    for (int d = 0; d < (int)cr[j].size(); ++d) evar[ebase[j] + d] = j;
  (void)ev_of;
  auto add_edge = [&](int e, int sg) {
    const int j = evar[e], d = e - ebase[j], i = erow[e];
    const int b = vbase + slot(i, pos[e]);
    rc[(size_t)rg(j, d) * 32 + b % 32] += sg;
    wc[(size_t)wg(j, d) * 16 + b % 16] += sg;
    auto& v = crow[rg(j, d)];
    auto it = std::find_if(v.begin(), v.end(), [&](const std::pair<int, int>& x) { return x.first == i; });
    if (sg > 0) {
      if (it == v.end()) {
        v.push_back({i, 1});
        cc[(size_t)rg(j, d) * 32 + (i + 1) % 32]++;
      } else {
        it->second++;
      }
    } else {
      if (--it->second == 0) {
        cc[(size_t)rg(j, d) * 32 + (i + 1) % 32]--;
        v.erase(it);
      }
    }
  };
  for (int e = 0; e < E; ++e) add_edge(e, +1);
  auto cost_groups = [&](const std::vector<int>& R, const std::vector<int>& Wg) {
    long long s = 0;
    for (int g : R) s += gmax(&rc[(size_t)g * 32], 32) + (long long)wcs * gmax(&cc[(size_t)g * 32], 32);
    for (int g : Wg) s += (long long)wst * gmax(&wc[(size_t)g * 16], 16);
    return s;
  };
  auto report = [&](const char* tag) {
    long long r = 0, w = 0, c = 0;
    int nr = 0, nw = 0;
    for (int g = 0; g < NRG; ++g) {
      const int a = gmax(&rc[(size_t)g * 32], 32);
      if (a) { r += a; ++nr; }
      c += gmax(&cc[(size_t)g * 32], 32);
    }
    for (int g = 0; g < NWG; ++g) {
      const int a = gmax(&wc[(size_t)g * 16], 16);
      if (a) { w += a; ++nw; }
    }
    printf("%s layout %c: cs %lld v_read %lld (%d groups) v_store %lld (%d groups) -> extra read %lld store %lld\n",
           tag, layout, c, r, nr, w, nw, r - nr, w - nw);
  };
  report("start");
  // degree classes for lane swaps: slots k < D3K hold degree-3 variables
  std::vector<int> cls3, cls4;
  for (int j = 0; j < n; ++j) (lane[j] / TB < D3K ? cls3 : cls4).push_back(j);
  for (long long it = 0; it < iters; ++it) {
    const double T = 0.5 * (1.0 - (double)it / iters);
    if ((double)(rnd() % 1000000) / 1e6 < lane_frac) {
      auto& cl = (rnd() & 1) ? cls3 : cls4;
      const int a = cl[rnd() % cl.size()], b = cl[rnd() % cl.size()];
      if (a == b || cr[a].size() != cr[b].size()) continue;
      std::vector<int> R, Wg;
      for (int x : {a, b})
        for (int d = 0; d < (int)cr[x].size(); ++d) {
          R.push_back(rg(x, d));
          Wg.push_back(wg(x, d));
        }
      auto uniq = [](std::vector<int>& v) {
        std::sort(v.begin(), v.end());
        v.erase(std::unique(v.begin(), v.end()), v.end());
      };
      // after the swap the groups are the same set (a takes b's lane and vice versa)
      uniq(R);
      uniq(Wg);
      const long long before = cost_groups(R, Wg);
      for (int x : {a, b})
        for (int d = 0; d < (int)cr[x].size(); ++d) add_edge(ebase[x] + d, -1);
      std::swap(lane[a], lane[b]);
      for (int x : {a, b})
        for (int d = 0; d < (int)cr[x].size(); ++d) add_edge(ebase[x] + d, +1);
      const long long dl = cost_groups(R, Wg) - before;
      if (!(dl <= 0 || (T > 0 && (double)(rnd() % 1000000) / 1e6 < std::exp(-(double)dl / T)))) {
        for (int x : {a, b})
          for (int d = 0; d < (int)cr[x].size(); ++d) add_edge(ebase[x] + d, -1);
        std::swap(lane[a], lane[b]);
        for (int x : {a, b})
          for (int d = 0; d < (int)cr[x].size(); ++d) add_edge(ebase[x] + d, +1);
      }
    } else {
      const int i = (int)(rnd() % (uint64_t)m);
      const int pa = (int)(rnd() % RW), pb = (int)(rnd() % RW);
      if (pa == pb) continue;
      const int ea = at[i][pa], eb = at[i][pb];
      if (ea < 0 && eb < 0) continue;
      std::vector<int> R, Wg;
      for (int e : {ea, eb})
        if (e >= 0) {
          R.push_back(rg(evar[e], e - ebase[evar[e]]));
          Wg.push_back(wg(evar[e], e - ebase[evar[e]]));
        }
      std::sort(R.begin(), R.end());
      R.erase(std::unique(R.begin(), R.end()), R.end());
      std::sort(Wg.begin(), Wg.end());
      Wg.erase(std::unique(Wg.begin(), Wg.end()), Wg.end());
      const long long before = cost_groups(R, Wg);
      for (int e : {ea, eb})
        if (e >= 0) add_edge(e, -1);
      if (ea >= 0) pos[ea] = pb;
      if (eb >= 0) pos[eb] = pa;
      for (int e : {ea, eb})
        if (e >= 0) add_edge(e, +1);
      const long long dl = cost_groups(R, Wg) - before;
      if (dl <= 0 || (T > 0 && (double)(rnd() % 1000000) / 1e6 < std::exp(-(double)dl / T))) {
        at[i][pa] = eb;
        at[i][pb] = ea;
      } else {
        for (int e : {ea, eb})
          if (e >= 0) add_edge(e, -1);
        if (ea >= 0) pos[ea] = pa;
        if (eb >= 0) pos[eb] = pb;
        for (int e : {ea, eb})
          if (e >= 0) add_edge(e, +1);
      }
    }
    if (it % (iters / 4 + 1) == 0 && it) report("  ...");
  }
  report("final");
  return 0;
}
