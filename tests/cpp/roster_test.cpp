// Host test of the co-residency roster (uasl_motion_estimation_amd/csrc/roster.hpp):
// the same protocol code the kernels run, over std atomics, with threads as
// workgroups -- some dispatched late, after the decider's close.  Checks, for
// the three launch shapes that use it:
//   persistent  (scale_lm_kernel): every workgroup joins, the first joiner
//               decides; units of every phase dealt over the participants,
//               the last arrival of a phase publishes the next one;
//   workers     (cam_solve_kernel<2>): block 0 decides without joining, the
//               workers join; P = 0 makes block 0 do every unit itself;
//   assemblers  (cam_solve_kernel<0/1> fused): a participant does its first
//               unit before it knows P, then strides by P.
// Invariants: every unit of every phase runs exactly once, late workgroups
// run nothing, nothing waits for a workgroup that has not joined, and the
// count equals the on-time joins.  Exit status 0 = pass.
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <thread>
#include <vector>

#include "../../uasl_motion_estimation_amd/csrc/roster.hpp"

namespace {

struct HostOps {
  static unsigned fetch_add(unsigned* p, unsigned v) { return __atomic_fetch_add(p, v, __ATOMIC_SEQ_CST); }
  static unsigned fetch_or(unsigned* p, unsigned v) { return __atomic_fetch_or(p, v, __ATOMIC_SEQ_CST); }
  static unsigned fetch_max(unsigned* p, unsigned v) {
    unsigned cur = __atomic_load_n(p, __ATOMIC_SEQ_CST);
    while (cur < v && !__atomic_compare_exchange_n(p, &cur, v, false, __ATOMIC_SEQ_CST, __ATOMIC_SEQ_CST)) {
    }
    return cur;
  }
  static unsigned load(const unsigned* p) { return __atomic_load_n(p, __ATOMIC_SEQ_CST); }
  static void store(unsigned* p, unsigned v) { __atomic_store_n(p, v, __ATOMIC_SEQ_CST); }
  static long long now() {  // 100 MHz ticks, as s_memrealtime
    return std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now().time_since_epoch())
               .count() / 10;
  }
  static void pause() { std::this_thread::yield(); }
};

int failures = 0;
#define CHECK(cond, ...)                  \
  do {                                    \
    if (!(cond)) {                        \
      std::fprintf(stderr, __VA_ARGS__);  \
      std::fprintf(stderr, "\n");         \
      ++failures;                         \
    }                                     \
  } while (0)

constexpr long long kWindow = 2000000;  // close window for the test: 20 ms (threads start within it)
constexpr int kLateMs = 200;            // late workgroups start this long after the launch

// Persistent grid: G workgroups, `late` of them dispatched after the close.
void persistent(int G, int late, int units, int phases) {
  unsigned roster[2] = {0, 0};
  std::atomic<unsigned> epoch{0};
  std::vector<std::atomic<int>> runs(units * phases);
  for (auto& r : runs) r = 0;
  std::atomic<unsigned> arrivals{0};
  std::atomic<int> participants{0}, late_work{0};
  auto wg = [&](bool is_late) {
    if (is_late) std::this_thread::sleep_for(std::chrono::milliseconds(kLateMs));
    int pid = me_roster::join<HostOps>(roster, (unsigned)G), np = 0;
    if (pid == 0)
      np = (int)me_roster::close<HostOps>(roster, (unsigned)G, kWindow);
    else if (pid > 0)
      np = me_roster::count<HostOps>(roster, 1L << 30);
    if (pid < 0) return;
    if (is_late) late_work++;
    participants++;
    for (int ph = 0; ph < phases; ++ph) {
      for (int u = pid; u < units; u += np) {
        runs[ph * units + u]++;
        if (arrivals.fetch_add(1) == (unsigned)units - 1) {  // last arrival: the phase's control
          arrivals = 0;
          epoch = (unsigned)ph + 1;
        }
      }
      long spins = 0;
      while (epoch.load() <= (unsigned)ph) {
        std::this_thread::yield();
        if (++spins > (1L << 28)) {
          CHECK(false, "persistent G=%d late=%d: a participant waited for ever at phase %d", G, late, ph);
          return;
        }
      }
    }
  };
  std::vector<std::thread> th;
  for (int i = 0; i < G; ++i) th.emplace_back(wg, i >= G - late);
  for (auto& t : th) t.join();
  for (int i = 0; i < units * phases; ++i)
    CHECK(runs[i] == 1, "persistent G=%d late=%d: unit %d of phase %d ran %d times", G, late, i % units,
          i / units, runs[i].load());
  CHECK(late_work == 0, "persistent: a late workgroup took part");
  CHECK(participants == G - late, "persistent G=%d late=%d: %d participants", G, late, participants.load());
}

// Camera-solve workers: block 0 decides (does not join); `nw` workers, `late`
// of them late; block0_late: block 0 itself is dispatched after the workers
// gave up on it (they depend on it, so they abandon the roster and block 0
// works alone).
void workers(int nw, int late, int units, int steps, bool close_now, bool block0_late = false) {
  unsigned roster[2] = {0, 0};
  std::vector<std::atomic<int>> runs(units * steps);
  for (auto& r : runs) r = 0;
  std::atomic<unsigned> step{0}, done{0};
  std::atomic<int> joined{0};
  int np0 = -1;
  auto block0 = [&]() {
    if (block0_late) std::this_thread::sleep_for(std::chrono::milliseconds(kLateMs));
    np0 = me_roster::close<HostOps>(roster, (unsigned)nw, close_now ? 0 : kWindow);
    for (int J = 0; J < steps; ++J) {
      if (np0 == 0) {
        for (int u = 0; u < units; ++u) runs[J * units + u]++;
      } else {
        step = (unsigned)J + 1;  // publish step J
        long spins = 0;
        while (done.load() < (unsigned)np0 * (J + 1)) {
          std::this_thread::yield();
          if (++spins > (1L << 28)) {
            CHECK(false, "workers: block 0 waited for ever at step %d", J);
            step = 1u << 30;
            return;
          }
        }
      }
    }
    step = 1u << 30;
  };
  auto worker = [&](bool is_late) {
    if (is_late) std::this_thread::sleep_for(std::chrono::milliseconds(kLateMs));
    const int pid = me_roster::join<HostOps>(roster, 0u);
    if (pid < 0) return;
    const int np = me_roster::count_or_abandon<HostOps>(roster, kWindow * 2);
    if (pid >= np) return;  // abandoned: block 0 works alone
    joined++;
    for (int J = 0; J < steps; ++J) {
      while (step.load() < (unsigned)J + 1) std::this_thread::yield();
      if (step.load() >= (1u << 30)) return;
      for (int u = pid; u < units; u += np) runs[J * units + u]++;
      done++;
    }
  };
  std::vector<std::thread> th;
  th.emplace_back(block0);
  for (int i = 0; i < nw; ++i) th.emplace_back(worker, i >= nw - late);
  for (auto& t : th) t.join();
  for (int i = 0; i < units * steps; ++i)
    CHECK(runs[i] == 1, "workers nw=%d late=%d now=%d: tile %d of step %d ran %d times", nw, late, (int)close_now,
          i % units, i / units, runs[i].load());
  CHECK(np0 == joined.load(), "workers: count %d vs %d joined", np0, joined.load());
  if (block0_late) CHECK(np0 == 0, "workers: block 0 late, count %d (the workers should have abandoned)", np0);
  else if (!close_now) CHECK(np0 == nw - late, "workers nw=%d late=%d: count %d", nw, late, np0);
}

// Fused assemblers (CLAIM): assembler u claims unit u; block 0 waits the
// window for the count, then claims and does every unit still unclaimed.
// Several launches in a row on the same claim words (generations 1, 2, 3).
void assemblers(int na, int late, bool steal_now, bool block0_late = false) {
  std::vector<unsigned> words(na, 0u);
  for (unsigned gen = 1; gen <= 3; ++gen) {
    std::vector<std::atomic<int>> runs(na);
    for (auto& r : runs) r = 0;
    std::atomic<unsigned> cnt{0};
    std::atomic<bool> b0_done{false};
    auto block0 = [&]() {
      if (block0_late) std::this_thread::sleep_for(std::chrono::milliseconds(kLateMs));
      const long long t0 = HostOps::now();
      while (cnt.load() < (unsigned)na && HostOps::now() - t0 < (steal_now ? 0 : kWindow)) HostOps::pause();
      if (cnt.load() < (unsigned)na)
        for (int u = 0; u < na; ++u)
          if (me_roster::claim<HostOps>(&words[u], gen)) {
            runs[u]++;
            cnt++;
          }
      long spins = 0;
      while (cnt.load() < (unsigned)na) {
        std::this_thread::yield();
        if (++spins > (1L << 28)) {
          CHECK(false, "assemblers: block 0 waited for ever");
          return;
        }
      }
      b0_done = true;
    };
    auto asmwg = [&](int u, bool is_late) {
      if (is_late) std::this_thread::sleep_for(std::chrono::milliseconds(kLateMs));
      if (!me_roster::claim<HostOps>(&words[u], gen)) return;
      if (b0_done.load()) CHECK(false, "assemblers: unit %d claimed after block 0 went on", u);
      runs[u]++;
      cnt++;
    };
    std::vector<std::thread> th;
    th.emplace_back(block0);
    for (int i = 0; i < na; ++i) th.emplace_back(asmwg, i, i >= na - late);
    for (auto& t : th) t.join();
    for (int u = 0; u < na; ++u)
      CHECK(runs[u] == 1, "assemblers na=%d late=%d now=%d gen=%u: unit %d ran %d times", na, late, (int)steal_now,
            gen, u, runs[u].load());
  }
}

}  // namespace

int main() {
  persistent(8, 0, 20, 6);
  persistent(8, 3, 20, 6);
  persistent(16, 15, 37, 4);
  persistent(1, 0, 5, 3);
  workers(6, 0, 21, 5, false);
  workers(6, 4, 21, 5, false);
  workers(6, 6, 21, 5, false);   // no worker on time: block 0 does every tile
  workers(6, 0, 21, 5, true);    // closed at once: whoever joined by then
  workers(6, 0, 21, 5, false, true);  // block 0 held back: the workers abandon, block 0 alone
  workers(6, 2, 21, 5, false, true);
  assemblers(12, 0, false);
  assemblers(12, 5, false);
  assemblers(12, 12, false);
  assemblers(12, 0, true);
  assemblers(12, 0, false, true);  // block 0 held back: the assemblers do every unit
  assemblers(12, 7, false, true);
  if (failures) {
    std::fprintf(stderr, "roster_test: %d failures\n", failures);
    return 1;
  }
  std::printf("roster_test: ok\n");
  return 0;
}
