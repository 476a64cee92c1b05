# Diagnostic variant (scripts/build_mix_variant.sh): the loader-form quad solver's compute waves
# read their row indices and labels with wave-uniform (scalar) loads -- one per lane group --
# instead of per-lane vector loads.
import sys
p = sys.argv[1]; s = open(p).read()
i = s.index("  // ---- compute wave: quad's step, the late classes from the LDS ring ----")
j = s.index("#undef QL_STEP")
k = s[i:j]
def rep(old, new):
    global k
    assert k.count(old) == 1, old[:60]
    k = k.replace(old, new)
rep("""  int idxq[DEPTH], labq[DEPTH];""", """  int idxq[DEPTH], labq[DEPTH];
  // wave-uniform row of lane group qq at the fetch cursor (a scalar load), and the lane's pick
  auto fetch_row_u = [&]() -> int {
    const int base = fep * nv + fsb * Bv;
    const int bcu = min(Bv, nv - fsb * Bv);
    int rq[4];
#pragma unroll
    for (int qq = 0; qq < 4; ++qq) {
      const int b = MQ_WAVES * w + qq;
      rq[qq] = perms[__builtin_amdgcn_readfirstlane(base + (b < bcu ? b : 0))];
    }
    if (fst + 1 < total) {
      ++fst;
      if (++fsb == nbat) {
        fsb = 0;
        ++fep;
      }
    }
    return q == 0 ? rq[0] : q == 1 ? rq[1] : q == 2 ? rq[2] : rq[3];
  };
  auto label_u = [&](int row) -> int {        // row is constant over a lane group: 4 scalar loads
    int lq[4];
#pragma unroll
    for (int qq = 0; qq < 4; ++qq) lq[qq] = y[__builtin_amdgcn_readlane(row, 16 * qq)];
    return q == 0 ? lq[0] : q == 1 ? lq[1] : q == 2 ? lq[2] : lq[3];
  };""")
rep("""    const int row = fetch_row();
    labq[k] = y[row];""", """    const int row = fetch_row_u();
    labq[k] = label_u(row);""")
rep("""  for (int k = 0; k < DEPTH; ++k) idxq[k] = fetch_row();""", """  for (int k = 0; k < DEPTH; ++k) idxq[k] = fetch_row_u();""")
rep("""    labq[R_] = y[idxq[R_]];                                                                  \\
    QL_ISSUE(R_, idxq[R_]);                                                                  \\
    idxq[R_] = fetch_row();                                                                  \\""", """    labq[R_] = label_u(idxq[R_]);                                                            \\
    QL_ISSUE(R_, idxq[R_]);                                                                  \\
    idxq[R_] = fetch_row_u();                                                                \\""")
s = s[:i] + k + s[j:]
open(p, 'w').write(s)
