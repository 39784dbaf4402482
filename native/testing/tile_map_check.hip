// Host-side check of the four-wave GEMM's workgroup -> tile maps
// (kgs::w4::tile_of in native/kernels/gemm_w4.h): for every map and a set of
// tile grids, every (slice, tile) is produced by exactly one workgroup, and
// for the blocked maps the first wave's eight XCDs never share one B column
// block among more than four XCDs. Prints one line per case; exit 1 on error.
// Built and run by tests/test_gemm_tile_map.py (host only, no GPU).
#include <cstdio>
#include <set>
#include <tuple>
#include <vector>

#include "gemm_w4.h"

template <int X, bool SPLITK>
static int check(int ntm, int ntn, int nslice) {
  const int grid = ntm * ntn * nslice;
  std::set<std::tuple<int, int, int>> seen;
  for (int b = 0; b < grid; ++b) {
    int s, tm, tn;
    kgs::w4::tile_of<X, SPLITK>(b, grid, ntm, ntn, s, tm, tn);
    if (s < 0 || s >= nslice || tm < 0 || tm >= ntm || tn < 0 || tn >= ntn) {
      std::printf("FAIL X=%d %dx%dx%d: block %d -> out of range (%d,%d,%d)\n", X, ntm, ntn, nslice, b, s, tm, tn);
      return 1;
    }
    if (!seen.insert({s, tm, tn}).second) {
      std::printf("FAIL X=%d %dx%dx%d: tile (%d,%d,%d) twice\n", X, ntm, ntn, nslice, s, tm, tn);
      return 1;
    }
  }
  // sharing degree of wave 1 (the first min(256, grid) blocks; block b on XCD b % 8)
  int max_share = 0;
  if (!SPLITK) {
    const int w1 = grid < 256 ? grid : 256;
    for (int col = 0; col < ntn; ++col) {
      std::set<int> xcds;
      for (int b = 0; b < w1; ++b) {
        int s, tm, tn;
        kgs::w4::tile_of<X, SPLITK>(b, grid, ntm, ntn, s, tm, tn);
        if (tn == col) xcds.insert(b & 7);
      }
      if ((int)xcds.size() > max_share) max_share = (int)xcds.size();
    }
  }
  std::printf("ok X=%d grid %dx%d slices %d: bijection, wave-1 B-column sharing %d XCDs\n", X, ntm, ntn, nslice,
              max_share);
  return 0;
}

int main() {
  int bad = 0;
  const int grids[][2] = {{32, 16}, {16, 32}, {32, 32}, {16, 16}, {64, 64}, {13, 7}, {1, 1}, {3, 112}, {48, 24}};
  for (auto& g : grids) {
    bad |= check<0, false>(g[0], g[1], 1);
    bad |= check<8, false>(g[0], g[1], 1);
    bad |= check<10000000, false>(g[0], g[1], 1);
    bad |= check<20000000, false>(g[0], g[1], 1);
    bad |= check<30000000, false>(g[0], g[1], 1);
    bad |= check<40000000, false>(g[0], g[1], 1);
    bad |= check<40000008, false>(g[0], g[1], 1);
    bad |= check<0, true>(g[0], g[1], 4);
    bad |= check<0, true>(g[0], g[1], 3);
  }
  return bad;
}
