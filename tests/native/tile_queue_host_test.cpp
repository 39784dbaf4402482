// Slot-ownership rules of native/kernels/tile_queue.h, on the host (fake HIP):
// distinct streams -> distinct slots (no wrap at any count), per-thread
// default stream keyed by thread, captured launches get a fresh slot each plus
// a memset node, never reused, reserve exhaustion during capture -> nullptr
// (the one-shot grid), a slot per (device, stream).
#include <cstdio>
#include <set>
#include <thread>

#include "../../native/kernels/tile_queue.h"

// the zeroing kernel of tile_queue_zero.h, on the host: recorded like a memset
// (captured when the stream is capturing, applied otherwise)
namespace kgs {
hipError_t tq_zero_slot(int* slot, hipStream_t stream) { return hipMemsetAsync(slot, 0, sizeof(int) * TQ_INTS, stream); }
}  // namespace kgs

#define CHECK(c)                                                         \
  do {                                                                   \
    if (!(c)) {                                                          \
      std::printf("FAIL line %d: %s\n", __LINE__, #c);                   \
      return 1;                                                          \
    }                                                                    \
  } while (0)

static hipStream_t S(long i) { return (hipStream_t)(0x10000 + 16 * i); }

int main() {
  using namespace kgs;
  // 1. 300 distinct streams: 300 distinct, zeroed slots; the same stream again -> the same slot
  std::set<int*> seen;
  for (int i = 0; i < 300; ++i) {
    int* q = tile_queue(S(i));
    CHECK(q != nullptr);
    for (int j = 0; j < TQ_INTS; ++j) CHECK(q[j] == 0);
    CHECK(seen.insert(q).second);
  }
  CHECK(tile_queue(S(7)) == tile_queue(S(7)));
  CHECK(tile_queue_stats(0).stream_slots == 300);
  // free slots kept for captures: more than the reserve after the growth
  CHECK(tile_queue_stats(0).slots - 300 > TQ_RESERVE);
  // 2. hipStreamPerThread: one slot per thread
  int* mine = tile_queue(hipStreamPerThread);
  int* theirs = nullptr;
  std::thread t([&] { theirs = tile_queue(hipStreamPerThread); });
  t.join();
  CHECK(mine && theirs && mine != theirs && !seen.count(mine) && !seen.count(theirs));
  CHECK(tile_queue(hipStreamPerThread) == mine);
  // 3. captures: each a fresh slot with a memset recorded on the capture stream, never S(0)'s
  fakehip::capturing()[S(0)] = true;
  const size_t m0 = fakehip::memsets().size();
  int* c1 = tile_queue(S(0));
  int* c2 = tile_queue(S(0));
  CHECK(c1 && c2 && c1 != c2 && c1 != tile_queue(S(1)));
  CHECK(!seen.count(c1) && !seen.count(c2) && c1 != mine && c2 != mine);
  CHECK(fakehip::memsets().size() == m0 + 2);
  CHECK(fakehip::memsets()[m0].p == c1 && fakehip::memsets()[m0].captured && fakehip::memsets()[m0].n == 64);
  // 4. no allocation during a capture: exhaust the reserve -> nullptr, counted
  const int mallocs = fakehip::mallocs();
  int got = 0;
  while (tile_queue(S(0)) != nullptr) ++got;
  CHECK(got > 0 && fakehip::mallocs() == mallocs);
  CHECK(tile_queue_stats(0).fallbacks == 1);
  fakehip::capturing()[S(0)] = false;
  // eager S(0) keeps its own slot (taken before the capture) ...
  CHECK(seen.count(tile_queue(S(0))));
  // ... and a new stream outside the capture grows the pool again
  int* fresh = tile_queue(S(1000));
  CHECK(fresh != nullptr && fakehip::mallocs() == mallocs + 1);
  // 5. a stream on device 1 gets device 1's pool (its own slot)
  fakehip::stream_dev()[S(2000)] = 1;
  int* d1 = tile_queue(S(2000));
  CHECK(d1 && tile_queue_stats(1).stream_slots == 1 && tile_queue_stats(0).stream_slots == 303);
  CHECK(fakehip::cur_dev() == 0);  // restored after allocating on device 1
  // 6. allocation failure on a fresh pool -> nullptr, not a crash
  fakehip::malloc_budget() = 0;
  fakehip::stream_dev()[S(3000)] = 2;
  CHECK(tile_queue(S(3000)) == nullptr && tile_queue_stats(2).fallbacks == 1);
  // 7. growth never touches a caller's stream: every chunk memset and every
  // sync went to a pool-private stream
  std::set<hipStream_t> priv(fakehip::created().begin(), fakehip::created().end());
  CHECK(priv.size() == 3);  // one per device that tried to grow (device 2: allocation then failed)
  // ... each created at the highest priority: its own hardware-queue pool, never a caller's queue
  CHECK(fakehip::priorities().size() == 3);
  for (int pr : fakehip::priorities()) CHECK(pr == -1);
  for (const auto& m : fakehip::memsets())
    CHECK(m.n == 64 ? !priv.count(m.s) : (priv.count(m.s) && !m.captured));
  CHECK(!fakehip::syncs().empty());
  for (hipStream_t s : fakehip::syncs()) CHECK(priv.count(s));
  // 8. captures that drain the reserve are refilled by the next eager call of
  // an already-known stream, not only by a new stream
  fakehip::malloc_budget() = 1 << 30;
  fakehip::capturing()[S(5)] = true;
  while (tile_queue(S(5)) != nullptr) {
  }
  const long fb = tile_queue_stats(0).fallbacks;
  fakehip::capturing()[S(5)] = false;
  const int mallocs2 = fakehip::mallocs();
  CHECK(seen.count(tile_queue(S(5))));  // its own slot, and the pool grew
  CHECK(fakehip::mallocs() == mallocs2 + 1);
  fakehip::capturing()[S(5)] = true;
  CHECK(tile_queue(S(5)) != nullptr && tile_queue_stats(0).fallbacks == fb);
  fakehip::capturing()[S(5)] = false;
  // 9. the quiescent-pool invariant: all zero; a stray word anywhere (here the
  // padding of a stream's slot) is found, with its value
  long chk[TQ_CHECK_OUT];
  CHECK(tile_queue_check(0, chk) == 0 && chk[0] == 0 && chk[1] == 0 && chk[3] == -1);
  int* victim = tile_queue(S(7));
  victim[12] = -792735554;  // 0xd0bed0be
  victim[3] = 5;
  CHECK(tile_queue_check(0, chk) == 0 && chk[0] == 1 && chk[1] == 2 && chk[2] == 5);
  CHECK(chk[4] == (long)(uintptr_t)victim && chk[5 + 3] == 5 && chk[5 + 12] == -792735554 && chk[5] == 0);
  victim[12] = victim[3] = 0;
  CHECK(tile_queue_check(0, chk) == 0 && chk[1] == 0);
  // 10. a kernel's impossible-ticket flag (padding word TQ_ERR) is counted separately
  victim[TQ_ERR] = (int)0x80000123;
  CHECK(tile_queue_check(0, chk) == 0 && chk[0] == 1 && chk[5 + TQ_INTS] == 1);
  victim[TQ_ERR] = 0;
  CHECK(tile_queue_check(0, chk) == 0 && chk[0] == 0 && chk[5 + TQ_INTS] == 0);
  // 11. a failed growth backs off: the next TQ_GROW_BACKOFF eager calls do not
  // retry hipMalloc / stream creation, then it is tried again
  fakehip::stream_dev()[S(4000)] = 3;
  fakehip::malloc_budget() = 0;
  CHECK(tile_queue(S(4000)) == nullptr && tile_queue_stats(3).grow_failures == 1);
  fakehip::malloc_budget() = 1 << 30;
  const int mallocs3 = fakehip::mallocs();
  for (int i = 0; i < tq_detail::TQ_GROW_BACKOFF; ++i) CHECK(tile_queue(S(4000)) == nullptr);
  CHECK(fakehip::mallocs() == mallocs3 && tile_queue_stats(3).fallbacks == 1 + tq_detail::TQ_GROW_BACKOFF);
  CHECK(tile_queue(S(4000)) != nullptr && fakehip::mallocs() == mallocs3 + 1);
  std::printf("tile_queue host test: OK (%ld slots on device 0)\n", tile_queue_stats(0).slots);
  return 0;
}
