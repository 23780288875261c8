// Host-only evaluator of engine-3 LDS layouts (development tool, no GPU):
// builds the decoder's slot map / check labels / edge table exactly as
// qldpc_bp_create does and counts the extra LDS-array cycles of one variable
// phase (CS gathers and v2c stores) under the bank model of MI355X_MICROARCH.md.
//   hipcc -O2 -I include tools/dev/layout_eval.cpp -o /tmp/layout_eval \
//     -Lqldpc_fault_tolerance_amd -lqldpc_hip && /tmp/layout_eval m n csr.bin prec TB VPL
#include "../../qldpc_fault_tolerance_amd/csrc/qldpc_hip.hip"

#include <cstdio>

static int store_extra(const std::vector<uint32_t>& vchk, int TB, int VPL, int DM, int tsize, int vbase_dw) {
  const int sg = tsize == 4 ? 32 : 16, nb = tsize == 4 ? 32 : 16, free_way = tsize == 4 ? 2 : 1;
  int extra = 0;
  for (int k = 0; k < VPL; ++k)
    for (int d = 0; d < DM; ++d)
      for (int h0 = 0; h0 < TB; h0 += sg) {
        int cnt[32] = {0};
        for (int t = h0; t < h0 + sg && t < TB; ++t) {
          const uint32_t e = vchk[((size_t)k * DM + d) * TB + t];
          if (e == 0) continue;
          const int slot = (int)(e >> 16);
          const int u = tsize == 4 ? vbase_dw + slot : vbase_dw / 2 + slot;
          cnt[u % nb]++;
        }
        int mx = 0;
        for (int b = 0; b < nb; ++b) mx = std::max(mx, cnt[b]);
        extra += std::max(0, (mx + free_way - 1) / free_way - 1);
      }
  return extra;
}

int main(int argc, char** argv) {
  if (argc < 7) return 1;
  const int m = atoi(argv[1]), n = atoi(argv[2]);
  FILE* f = fopen(argv[3], "rb");
  std::vector<int32_t> rp(m + 1), ci;
  if (fread(rp.data(), 4, m + 1, f) != (size_t)m + 1) return 2;
  ci.resize(rp[m]);
  if (fread(ci.data(), 4, rp[m], f) != (size_t)rp[m]) return 2;
  fclose(f);
  const int prec = atoi(argv[4]), TB = atoi(argv[5]), VPL = atoi(argv[6]);
  qldpc_graph* g = nullptr;
  if (qldpc_graph_create(0, m, n, rp.data(), ci.data(), &g)) return 3;
  const int tsize = prec == 32 ? 4 : 8, DM = 4;
  const int nch = (std::max(1, g->max_row) * tsize + 15) / 16;
  const int vslots = (1 + m * nch) * (16 / tsize);
  std::vector<int32_t> order;
  for (int pass = 0; pass < 2; ++pass)
    for (int j = 0; j < n; ++j)
      if (((int)g->col_rows[j].size() <= 3) == (pass == 0)) order.push_back(j);
  std::vector<int32_t> slot_var((size_t)VPL * TB, -1);
  for (int j = 0; j < n; ++j) slot_var[j] = order[j];
  const int vbase_dw = (int)(r_layout(3, vslots, m, tsize).v / 4);
  std::vector<uint32_t> v0, v1, v2;
  build_slot_edges(g, TB, VPL, DM, tsize, nch, slot_var, v0, -1);
  build_slot_edges(g, TB, VPL, DM, tsize, nch, slot_var, v1, vbase_dw);
  int gb = 0, ga = 0;
  std::vector<int> lab = label_checks(g, slot_var, TB, VPL, DM, tsize, &gb, &ga);
  build_slot_edges(g, TB, VPL, DM, tsize, nch, slot_var, v2, vbase_dw, lab);
  printf("m=%d n=%d prec=%d TB=%d VPL=%d nch=%d\n", m, n, prec, TB, VPL, nch);
  printf("gather extra/pass: identity %d, labelled %d\n", gb, ga);
  printf("store extra/pass: ascending %d, greedy %d, labelled+greedy %d (of %d store wave-instr groups)\n",
         store_extra(v0, TB, VPL, DM, tsize, vbase_dw), store_extra(v1, TB, VPL, DM, tsize, vbase_dw),
         store_extra(v2, TB, VPL, DM, tsize, vbase_dw), VPL * DM * TB / (tsize == 4 ? 32 : 16));
  return 0;
}
