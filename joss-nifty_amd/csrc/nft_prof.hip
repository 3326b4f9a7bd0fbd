// Per-launch kernel timing with HIP events (bench.py roofline probe).
//
// nft_prof_begin(cap) arms the profiler; every hot-path launch site calls
// prof_mark(stream, label) just before its kernel, recording an event on the
// launch stream; nft_prof_end records a closing event, waits for it and
// returns, per launch, the label and the elapsed milliseconds between its
// event and the next one (= that kernel's duration when launches are queued
// back to back).  Not thread-safe; not for use inside HIP graph capture.
#include <string>
#include <vector>

#include "nft_api_internal.hpp"

namespace nft {

bool g_prof_on = false;
static std::vector<hipEvent_t> g_ev;
static std::vector<std::string> g_lab;
static size_t g_cap = 0;
// the first failed event call of a profiling window (reported by nft_prof_end)
static hipError_t g_err = hipSuccess;

void prof_mark_impl(hipStream_t s, const char* label) {
  if (g_lab.size() >= g_cap) return;
  hipEvent_t e;
  // no system-scope release: the default fence writes back L2 and would perturb
  // the next kernel's cache state
  hipError_t st = hipEventCreateWithFlags(&e, hipEventDisableSystemFence);
  if (st == hipSuccess) {
    st = hipEventRecord(e, s);
    if (st != hipSuccess) (void)hipEventDestroy(e);
  }
  if (st != hipSuccess) {
    if (g_err == hipSuccess) g_err = st;
    return;
  }
  g_ev.push_back(e);
  g_lab.push_back(label);
}

}  // namespace nft

using namespace nft;

extern "C" {

int nft_prof_begin(int capacity) {
  hipError_t st = hipSuccess;
  for (auto e : g_ev) {
    const hipError_t d = hipEventDestroy(e);
    if (st == hipSuccess) st = d;
  }
  g_ev.clear();
  g_err = hipSuccess;
  g_lab.clear();
  g_cap = capacity > 0 ? (size_t)capacity : 0;
  g_prof_on = g_cap > 0;
  NFT_HIP_CHECK(st);
  return NFT_OK;
}

int nft_prof_end(hipStream_t stream, float* ms, int cap, int* n) {
  g_prof_on = false;
  const int m = (int)g_ev.size();
  *n = 0;
  if (m == 0) {
    NFT_HIP_CHECK(g_err);
    return NFT_OK;
  }
  hipEvent_t last;
  NFT_HIP_CHECK(hipEventCreate(&last));
  NFT_HIP_CHECK(hipEventRecord(last, stream));
  NFT_HIP_CHECK(hipEventSynchronize(last));
  int k = 0;
  for (int i = 0; i < m && k < cap; ++i, ++k) {
    float t = 0.f;
    NFT_HIP_CHECK(hipEventElapsedTime(&t, g_ev[i], i + 1 < m ? g_ev[i + 1] : last));
    ms[k] = t;
  }
  *n = k;
  NFT_HIP_CHECK(hipEventDestroy(last));
  NFT_HIP_CHECK(g_err);  // a mark that could not be recorded: the times above skip it
  return NFT_OK;
}

const char* nft_prof_label(int i) {
  return (i >= 0 && i < (int)g_lab.size()) ? g_lab[i].c_str() : "";
}

}  // extern "C"
