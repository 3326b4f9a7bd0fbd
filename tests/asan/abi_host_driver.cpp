// Host-side checks of the C ABI under AddressSanitizer (SURVEY.md §5,
// "race detection / sanitizers"): the library's host code -- argument
// validation, workspace sizing, plan arithmetic, error formatting -- built
// with -fsanitize=address for the host (GPU code untouched; GPU ASan is not
// available on the target pool) and driven through every entry point whose
// work finishes on the host.  No call here reaches the device: the invalid
// arguments are rejected before any launch.  Exit code 0 = every check held
// and ASan reported nothing.
#include <cstdio>
#include <cstring>
#include <vector>

#include "nifty_amd.h"

static int fails = 0;
#define CHECK(c)                                                   \
  do {                                                             \
    if (!(c)) {                                                    \
      std::fprintf(stderr, "FAILED %s:%d: %s\n", __FILE__, __LINE__, #c); \
      ++fails;                                                     \
    }                                                              \
  } while (0)

static bool err_mentions(const char* s) {
  const char* e = nft_last_error();
  return e && std::strstr(e, s) != nullptr;
}

int main() {
  // workspace sizing over many shapes / axis sets (parse_axes, half_shape)
  for (int nd = 1; nd <= 3; ++nd) {
    for (int64_t n : {1, 2, 7, 16, 63, 1024, 2048}) {
      std::vector<int64_t> shape(nd, n);
      std::vector<int> axes;
      for (int a = 0; a < nd; ++a) axes.push_back(a);
      for (int dt = 0; dt < 2; ++dt) {
        size_t b1 = 0, b2 = 0;
        CHECK(nft_hartley_workspace(nd, shape.data(), nd, axes.data(), dt, &b1) == NFT_OK);
        CHECK(nft_hartley_fused_workspace(nd, shape.data(), nd, axes.data(), dt, &b2) == NFT_OK);
        CHECK(b2 >= b1);
        // negative axes and repeated axes are folded, not overrun
        std::vector<int> neg(axes.size());
        for (size_t i = 0; i < axes.size(); ++i) neg[i] = axes[i] - nd;
        size_t b3 = 0;
        CHECK(nft_hartley_workspace(nd, shape.data(), nd, neg.data(), dt, &b3) == NFT_OK && b3 == b1);
      }
    }
  }
  {
    int64_t shape[2] = {16, 16};
    int bad_axes[2] = {0, 5};
    size_t b = 0;
    CHECK(nft_hartley_workspace(2, shape, 2, bad_axes, 0, &b) == NFT_ERR_ARG && err_mentions("axis 5"));
    CHECK(nft_hartley_workspace(0, shape, 0, bad_axes, 0, &b) == NFT_ERR_ARG && err_mentions("ndim"));
    int64_t empty[2] = {16, 0};
    int axes[2] = {0, 1};
    CHECK(nft_hartley_workspace(2, empty, 2, axes, 0, &b) == NFT_ERR_ARG && err_mentions("empty"));
    // the fused transform rejects the same geometry before touching buffers
    CHECK(nft_hartley_fused(nullptr, nullptr, nullptr, 2, shape, 2, bad_axes, 0, 0, 1.0, nullptr, 0, nullptr) ==
          NFT_ERR_ARG);
  }
  // reduction / CG / amplitude / bin sizing
  for (int64_t n : {1LL, 255LL, 256LL, 4194304LL, 4821009LL}) {
    CHECK(nft_reduce_workspace(n) > 0);
    CHECK(nft_cg_dd_blocks(n) >= 1);
  }
  for (int64_t B : {3LL, 1024LL, 313847LL}) {
    CHECK(nft_amp_workspace(B) >= (size_t)(3 * B) * sizeof(double));
    CHECK(nft_amp_forward_buf(B) == 5 * (B - 2) + 4 * B);
  }
  CHECK(nft_bin_chunk() > 0);
  // two-phase amplitude kernels: tile counts (host arithmetic) and argument checks
  CHECK(nft_amp2_tiles(313847, 4, 0) == 307);   // 1024-bin tiles, whatever the batch
  CHECK(nft_amp2_tiles(313847, 1, 2) == 307);
  CHECK(nft_amp2_tiles(1197363, 8, 1) == 1170);  // C5
  CHECK(nft_amp2_tiles(313847, 300, 0) == 0);    // more RHS than arrival counters
  CHECK(nft_amp2_tiles(2, 1, 0) == 0);
  CHECK(nft_amp2_tab_size(2) == 0);
  CHECK(nft_amp2_tab_size(313847) == 5 * 313856 + 16 * 307);  // 5 padded scans + 16 rows of 307 tiles
  CHECK(nft_amp2_prepare(nullptr, nullptr, 0, nullptr, nullptr) == NFT_ERR_ARG && err_mentions("nft_amp2_prepare"));
  {
    void* t[6] = {nullptr, nullptr, nullptr, nullptr, nullptr, nullptr};
    CHECK(nft_amp2_jvp(nullptr, nullptr, 0, t, nullptr, 0, nullptr, 0, 0, nullptr, 1, nullptr, nullptr, 0, 0.0, 0,
                       nullptr, nullptr) == NFT_ERR_ARG && err_mentions("nft_amp2_jvp"));
    void* o[6] = {nullptr, nullptr, nullptr, nullptr, nullptr, nullptr};
    CHECK(nft_amp2_vjp(nullptr, nullptr, 0, nullptr, 0, o, nullptr, nullptr, 0, 0.0, nullptr, 1, nullptr, nullptr, 0,
                       nullptr, 0, 0, 0, 0, nullptr, nullptr) == NFT_ERR_ARG && err_mentions("nft_amp2_vjp"));
  }
  // CG segment update: partial blocks outside the partial array
  CHECK(nft_cg_update_seg_batched(nullptr, nullptr, nullptr, nullptr, nullptr, 1 << 20, 1 << 20, 4, 0, 1.0,
                                  nullptr, nullptr, 8, 4, nullptr) == NFT_ERR_ARG &&
        err_mentions("partial blocks"));
  // amplitude forward: every invalid combination is rejected on the host
  {
    nft_amp_model m;
    std::memset(&m, 0, sizeof(m));
    m.B = 100;
    m.has_flex = 1;
    double dummy[8] = {0};
    nft_amp_const dc[2];
    CHECK(nft_amp_forward_batched(&m, dummy, dummy, nullptr, nullptr, nullptr, nullptr, 0, 1, dummy, 100, dummy,
                                  1000, dc, dummy, nullptr) == NFT_ERR_ARG);   // has_flex without spectrum
    m.has_flex = 0;
    CHECK(nft_amp_forward_batched(&m, dummy, dummy, nullptr, nullptr, nullptr, nullptr, 0, 1, dummy, 100, dummy,
                                  10, dc, dummy, nullptr) == NFT_ERR_ARG);     // buffer stride too small
    CHECK(nft_amp_forward_batched(nullptr, dummy, dummy, nullptr, nullptr, nullptr, nullptr, 0, 1, dummy, 100,
                                  dummy, 1000, dc, dummy, nullptr) == NFT_ERR_ARG);
    CHECK(err_mentions("nft_amp_forward_batched"));
  }
  // LOS: plan validation and the batched / per-vector-scale argument checks
  {
    nft_los_plan p;
    std::memset(&p, 0, sizeof(p));
    CHECK(nft_los_forward_ex(&p, nullptr, nullptr, 0, nullptr, nullptr, nullptr, 0, 1.0, 1, 0, 0, nullptr, 0,
                             nullptr) == NFT_ERR_ARG && err_mentions("invalid plan"));
    p.bh = 16;
    p.bw = 16;
    p.nbx = 1;
    p.nby = 1;
    p.nlos = 37;
    p.nseg = 5;
    CHECK(nft_los_quad_blocks(&p) == 10);
    CHECK(nft_los_workspace(&p) >= 5 * sizeof(double));
    CHECK(nft_los_forward_ex(&p, nullptr, nullptr, 0, nullptr, nullptr, nullptr, 0, 1.0, 0, 0, 0, nullptr, 0,
                             nullptr) == NFT_ERR_ARG);                          // nvec 0
    CHECK(nft_los_forward_ex(&p, nullptr, nullptr, -1, nullptr, nullptr, nullptr, 0, 1.0, 2, 0, 0, nullptr, 0,
                             nullptr) == NFT_ERR_ARG);                          // negative scale stride
    double q[4];
    CHECK(nft_los_forward_ex(&p, nullptr, nullptr, 0, nullptr, nullptr, nullptr, 0, 1.0, 2, 0, 0, q, 3,
                             nullptr) == NFT_ERR_ARG);                          // qstride < quad blocks
    CHECK(nft_los_forward_quad_batched(&p, nullptr, nullptr, nullptr, nullptr, nullptr, 0, 1.0, 9, 0, 0, q, 10,
                                       nullptr) == NFT_ERR_ARG);                // nvec > 8
    CHECK(nft_los_adjoint_ex(&p, nullptr, nullptr, nullptr, -5, nullptr, 0, 1.0, 1, 0, 0, nullptr) ==
          NFT_ERR_ARG && err_mentions("rowscale_stride"));
    CHECK(nft_los_forward_batched(&p, nullptr, nullptr, nullptr, nullptr, nullptr, 7, 1.0, 1, 0, 0, nullptr) ==
          NFT_ERR_ARG && err_mentions("bad dtype"));
  }
  // long error messages stay within the thread-local buffer
  {
    int64_t shape[1] = {8};
    int axes[1] = {-1234567890};
    size_t b = 0;
    CHECK(nft_hartley_workspace(1, shape, 1, axes, 0, &b) == NFT_ERR_ARG);
    CHECK(std::strlen(nft_last_error()) < 4096);
  }
  if (fails) {
    std::fprintf(stderr, "%d check(s) failed\n", fails);
    return 1;
  }
  std::printf("abi host checks: ok\n");
  return 0;
}
