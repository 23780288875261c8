// place_opt4.cpp — offline study (round 4): "layout C" for the m2s variable phase: every row is 8
// aligned 8-byte slots (slot = 8 lab + pos, pos < 8) holding its 7 edges' V slots AND its CS word at
// a per-row position cs(lab), i.e. the same 52 KiB image as the current 3 chunks + tail + CS array.
// Aligned rows make the bank of slot (lab, pos) = (c0 + 8 (lab mod 4) + pos) mod 32 for 32-lane
// reads, (c0 + 8 (lab mod 2) + pos) mod 16 for 16-lane stores: with the labels' classes balanced per
// lane group, conflict-free reads / stores / CS gathers are an edge colouring.  Annealing over
// label swaps (L), in-row position swaps including the CS position (P) on the exact lane-group
// model of qldpc_bp_lds_model.
//   g++ -O2 -o /tmp/place_opt4 tools/dev/place_opt4.cpp && /tmp/place_opt4 /tmp/hz.txt 20000000 PL [T0] [balance]
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
  // optional phase 0 (argv[5] = balance moves): label swaps minimising, per read group, the spread of
  // its rows' classes (lab mod 4) and, per store group, of (lab mod 2): sum of squared counts
  const long long bal_iters = argc > 5 ? atoll(argv[5]) : 0;
  if (bal_iters > 0) {
    std::vector<std::vector<int>> rc4(NR, std::vector<int>(4, 0)), wc2(NW, std::vector<int>(2, 0));
    auto bal_put = [&](int e, int sg) {
      const int l = lab[ed[e].row];
      rc4[rg(e)][l & 3] += sg;
      wc2[wg(e)][l & 1] += sg;
    };
    for (size_t e = 0; e < ed.size(); ++e) bal_put((int)e, +1);
    auto bcost = [&](const std::vector<int>& es) {
      long long v = 0;
      std::vector<int> gr, gw;
      for (int e : es) { gr.push_back(rg(e)); gw.push_back(wg(e)); }
      std::sort(gr.begin(), gr.end()); gr.erase(std::unique(gr.begin(), gr.end()), gr.end());
      std::sort(gw.begin(), gw.end()); gw.erase(std::unique(gw.begin(), gw.end()), gw.end());
      for (int g : gr) for (int q = 0; q < 4; ++q) v += (long long)rc4[g][q] * rc4[g][q];
      for (int g : gw) for (int q = 0; q < 2; ++q) v += (long long)wc2[g][q] * wc2[g][q];
      return v;
    };
    for (long long it = 0; it < bal_iters; ++it) {
      const int i1 = (int)(rnd() % (uint64_t)m), i2 = (int)(rnd() % (uint64_t)m);
      if (i1 == i2 || ((lab[i1] ^ lab[i2]) & 3) == 0) continue;
      std::vector<int> es = row_e[i1];
      es.insert(es.end(), row_e[i2].begin(), row_e[i2].end());
      const long long before = bcost(es);
      for (int e : es) bal_put(e, -1);
      std::swap(lab[i1], lab[i2]);
      for (int e : es) bal_put(e, +1);
      if (bcost(es) > before) {
        for (int e : es) bal_put(e, -1);
        std::swap(lab[i1], lab[i2]);
        for (int e : es) bal_put(e, +1);
      }
    }
    long long worst = 0, sumsq = 0;
    for (int g = 0; g < NR; ++g) for (int q = 0; q < 4; ++q) { worst = std::max<long long>(worst, rc4[g][q]); sumsq += (long long)rc4[g][q] * rc4[g][q]; }
    printf("balance: max class count per read group %lld, sum sq %lld\n", worst, sumsq);
    // re-seat every edge and the CS words under the new labels
    for (auto& g : R) g.init();
    for (auto& g : W) g.init();
    for (auto& g : C) g.init();
    csm.clear();
    for (size_t e = 0; e < ed.size(); ++e) put((int)e, +1);
  }
  // optional phase 1 (argv[6] = 1): per label class (lab mod 4), a proper 8-edge-colouring of the
  // bipartite multigraph rows x read groups (Konig: max degree 8 after balancing) by alternating-path
  // recolouring; colour = the edge's position in its row, the row's free colour = its CS position.
  // Conflict-free V-slot reads by construction (when every group holds <= 8 rows of each class).
  if (argc > 6 && atoi(argv[6]) == 1) {
    const int NC = 8;
    // colour tables: at_row[i][c] = edge or -1, at_grp[g][c] = edge or -1 (per class: groups are shared
    // across classes, so index by (class, group))
    std::vector<std::vector<int>> at_row(m, std::vector<int>(NC, -1));
    std::vector<std::vector<int>> at_grp((size_t)NR * 4, std::vector<int>(NC, -1));
    std::vector<int> col(ed.size(), -1);
    auto gkey = [&](int e) { return (size_t)rg(e) * 4 + (lab[ed[e].row] & 3); };
    int failed = 0;
    for (size_t e0 = 0; e0 < ed.size(); ++e0) {
      const int e = (int)e0, i = ed[e].row;
      const size_t gk = gkey(e);
      int a = -1, b = -1;
      for (int c2 = 0; c2 < NC && a < 0; ++c2)
        if (at_row[i][c2] < 0) a = c2;
      for (int c2 = 0; c2 < NC && b < 0; ++c2)
        if (at_grp[gk][c2] < 0) b = c2;
      if (a < 0 || b < 0) { ++failed; continue; }
      if (at_grp[gk][a] >= 0) {
        // flip the a/b alternating path that starts at group gk with colour a
        std::vector<int> path;
        size_t g = gk;
        int row = -1;
        int cur = a;
        while (true) {
          const int pe = at_grp[g][cur];
          if (pe < 0) break;
          path.push_back(pe);
          row = ed[pe].row;
          const int nxt = cur == a ? b : a;
          const int qe = at_row[row][nxt];
          if (qe < 0) break;
          path.push_back(qe);
          g = gkey(qe);
          cur = a;  // from the group side we follow colour a again (a, b, a, b ...)
          (void)cur;
        }
        for (int pe : path) {  // unassign
          at_row[ed[pe].row][col[pe]] = -1;
          at_grp[gkey(pe)][col[pe]] = -1;
        }
        for (int pe : path) {  // swap a <-> b
          col[pe] = col[pe] == a ? b : a;
          at_row[ed[pe].row][col[pe]] = pe;
          at_grp[gkey(pe)][col[pe]] = pe;
        }
      }
      if (at_row[i][a] >= 0 || at_grp[gk][a] >= 0) { ++failed; continue; }
      col[e] = a;
      at_row[i][a] = e;
      at_grp[gk][a] = e;
    }
    // positions: colour = position; the CS word takes the row's free colour
    for (int i = 0; i < m; ++i) {
      for (int q = 0; q < 8; ++q) at[i][q] = -1;
      for (int e : row_e[i]) if (col[e] >= 0) { at[i][col[e]] = e; ed[e].ps = col[e]; }
      for (int e : row_e[i]) if (col[e] < 0) for (int q = 0; q < 8; ++q) if (at[i][q] == -1) { at[i][q] = e; ed[e].ps = q; break; }
      for (int q = 0; q < 8; ++q) if (at[i][q] == -1) { at[i][q] = -2; break; }
    }
    printf("colouring: %d edges left uncoloured\n", failed);
    // phase 2 (argv[7] = moves): Kempe-chain recolouring inside one class graph (swap colours a <-> b
    // along the alternating path through an edge): the colouring stays proper, so the reads stay
    // conflict-free, while the positions of the chain's edges and the free colour (CS position) of
    // its end rows change; accepted when CS + stores do not get worse (exact group costs)
    const long long kmoves = argc > 7 ? atoll(argv[7]) : 0;
    if (kmoves > 0) {
      std::vector<int> tr, tw;
      auto rebuild_at = [&](int i) {
        for (int q = 0; q < 8; ++q) at[i][q] = -1;
        for (int e : row_e[i]) { at[i][col[e]] = e; ed[e].ps = col[e]; }
        for (int q = 0; q < 8; ++q) if (at[i][q] == -1) { at[i][q] = -2; break; }
      };
      for (int i = 0; i < m; ++i) rebuild_at(i);
      for (auto& g : R) g.init();
      for (auto& g : W) g.init();
      for (auto& g : C) g.init();
      csm.clear();
      for (size_t e = 0; e < ed.size(); ++e) put((int)e, +1);
      long long acc = 0;
      for (long long it = 0; it < kmoves; ++it) {
        const int e0 = (int)(rnd() % (uint64_t)ed.size());
        const int a = col[e0];
        int b = (int)(rnd() % 7);
        if (b >= a) ++b;
        // collect the chain: from e0 walk both directions alternating a/b
        std::vector<int> chain{e0};
        for (int dir = 0; dir < 2; ++dir) {
          int e = e0;
          bool at_group = dir == 0;  // first step: across the group (dir 0) or the row (dir 1)
          int want = b;
          for (int guard = 0; guard < 4000; ++guard) {
            int nx = at_group ? at_grp[gkey(e)][want] : at_row[ed[e].row][want];
            if (nx < 0 || nx == e0) break;
            chain.push_back(nx);
            e = nx;
            at_group = !at_group;
            want = want == a ? b : a;
          }
        }
        std::sort(chain.begin(), chain.end());
        chain.erase(std::unique(chain.begin(), chain.end()), chain.end());
        if (chain.size() > 400) continue;
        // affected rows: rows of chain edges (all their edges' CS entries move with the CS position)
        std::vector<int> rows;
        for (int e : chain) rows.push_back(ed[e].row);
        std::sort(rows.begin(), rows.end());
        rows.erase(std::unique(rows.begin(), rows.end()), rows.end());
        std::vector<int> es;
        for (int i : rows) es.insert(es.end(), row_e[i].begin(), row_e[i].end());
        tr.clear();
        tw.clear();
        for (int e : es) { tr.push_back(rg(e)); tw.push_back(wg(e)); }
        auto cs_store = [&]() {
          std::sort(tr.begin(), tr.end()); tr.erase(std::unique(tr.begin(), tr.end()), tr.end());
          std::sort(tw.begin(), tw.end()); tw.erase(std::unique(tw.begin(), tw.end()), tw.end());
          double v = 0;
          for (int g : tr) v += C[g].cost() + R[g].cost();
          for (int g : tw) v += W[g].cost();
          return v;
        };
        const double before = cs_store();
        auto flip = [&]() {
          for (int e : es) put(e, -1);
          for (int e : chain) { at_row[ed[e].row][col[e]] = -1; at_grp[gkey(e)][col[e]] = -1; }
          for (int e : chain) col[e] = col[e] == a ? b : a;
          for (int e : chain) { at_row[ed[e].row][col[e]] = e; at_grp[gkey(e)][col[e]] = e; }
          for (int i : rows) rebuild_at(i);
          for (int e : es) put(e, +1);
        };
        flip();
        const double after = cs_store();
        if (after > before) flip(); else ++acc;
        if ((it + 1) % (kmoves / 5 > 0 ? kmoves / 5 : 1) == 0) {
          long long c2, r2, w2;
          totals(c2, r2, w2);
          printf("kempe %lld: cs %lld read %lld store %lld (accepted %lld)\n", it + 1, c2, r2, w2, acc);
          fflush(stdout);
        }
      }
    }
    for (auto& g : R) g.init();
    for (auto& g : W) g.init();
    for (auto& g : C) g.init();
    csm.clear();
    for (size_t e = 0; e < ed.size(); ++e) put((int)e, +1);
  }
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
