// Node-wide per-GPU share board (include/vgpu/board.h): fair-share charging of
// GPU time between the pods that time-share one physical device.
#include <algorithm>
#include "board.h"

#include <errno.h>
#include <stdio.h>
#include <fcntl.h>
#include <sys/file.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include "common.h"
#include "state.h"

namespace vgpu {

static_assert(sizeof(pthread_mutex_t) <= 64, "mutex must fit its 64-byte slot");

namespace {

void init_board(vgpu_board_t* b) {
  memset(b, 0, sizeof(*b));
  b->magic = VGPU_BOARD_MAGIC;
  b->version = VGPU_BOARD_VERSION;
  b->struct_size = (uint32_t)sizeof(*b);
  pthread_mutexattr_t a;
  pthread_mutexattr_init(&a);
  pthread_mutexattr_setpshared(&a, PTHREAD_PROCESS_SHARED);
  pthread_mutexattr_setrobust(&a, PTHREAD_MUTEX_ROBUST);
  pthread_mutex_init(&b->lock.m, &a);
  pthread_mutexattr_destroy(&a);
  b->last_ns = mono_ns();
  __atomic_store_n(&b->initialized, 1, __ATOMIC_RELEASE);
}

bool lock(vgpu_board_t* b) {
  int rc = pthread_mutex_lock(&b->lock.m);
  if (rc == EOWNERDEAD) {
    pthread_mutex_consistent(&b->lock.m);
    rc = 0;
  }
  return rc == 0;
}

void unlock(vgpu_board_t* b) { pthread_mutex_unlock(&b->lock.m); }

bool live(const vgpu_board_slot_t& s, uint64_t now) {
  return s.pid != 0 && s.active && now - s.heartbeat_ns < VGPU_BOARD_STALE_NS;
}

// Advance virtual time to `now` at the rate set by the active count of the
// previous interval, then recount (caller holds the lock).
void advance(vgpu_board_t* b, uint64_t now) {
  if (now > b->last_ns) {
    const int n = b->n_active > 1 ? b->n_active : 1;
    b->v += (double)(now - b->last_ns) / n;
    b->last_ns = now;
  }
  int n = 0;
  for (int i = 0; i < VGPU_BOARD_SLOTS; ++i) n += live(b->slot[i], now);
  b->n_active = n;
}

}  // namespace

vgpu_board_t* board_map(const char* path) {
  const size_t sz = sizeof(vgpu_board_t);
  int fd = open(path, O_RDWR | O_CREAT | O_CLOEXEC, 0666);
  if (fd < 0) {
    VLOG_WARN("cannot open share board %s: %s", path, strerror(errno));
    return nullptr;
  }
  flock(fd, LOCK_EX);
  // The layout version is part of the file name (limiter.cpp), so a board of
  // another layout is never expected here.  Only an empty file or a board
  // nobody finished initialising (magic 0: its creator died between ftruncate
  // and init, both under this flock) is (re)initialised.  Anything else that
  // does not match may be in use by a live process of another build, whose
  // robust mutex must not be wiped under it: refuse it (wall-time charging).
  struct {
    uint32_t magic, version, size;
    int32_t initialized;
  } hdr = {};
  struct stat stt;
  fstat(fd, &stt);
  const bool have_hdr = pread(fd, &hdr, sizeof hdr, 0) == (ssize_t)sizeof hdr;
  const bool blank = !have_hdr || (hdr.magic == 0 && hdr.initialized == 0);
  if (!blank && (hdr.magic != VGPU_BOARD_MAGIC || hdr.version != VGPU_BOARD_VERSION || hdr.size != sz ||
                 !hdr.initialized || (size_t)stt.st_size < sz)) {
    VLOG_WARN("share board %s has another layout (magic %#x version %u size %u); charging wall time", path,
              hdr.magic, hdr.version, hdr.size);
    flock(fd, LOCK_UN);
    close(fd);
    return nullptr;
  }
  if ((size_t)stt.st_size < sz && ftruncate(fd, (off_t)sz) != 0) {
    flock(fd, LOCK_UN);
    close(fd);
    return nullptr;
  }
  void* p = mmap(nullptr, sz, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
  if (p == MAP_FAILED) {
    flock(fd, LOCK_UN);
    close(fd);
    return nullptr;
  }
  auto* b = (vgpu_board_t*)p;
  if (blank) init_board(b);
  flock(fd, LOCK_UN);
  close(fd);
  return b;
}

int board_claim(vgpu_board_t* b, int pid, int host_pid, int limit_pct) {
  if (!b || !lock(b)) return -1;
  const uint64_t now = mono_ns();
  int got = -1;
  for (int i = 0; i < VGPU_BOARD_SLOTS && got < 0; ++i) {
    vgpu_board_slot_t& s = b->slot[i];
    // free, or abandoned (no heartbeat for 10 x the stale interval)
    if (s.pid == 0 || now - s.heartbeat_ns > 10 * VGPU_BOARD_STALE_NS) got = i;
  }
  if (got >= 0) {
    vgpu_board_slot_t& s = b->slot[got];
    memset(&s, 0, sizeof(s));
    s.pid = pid;
    s.host_pid = host_pid;
    s.limit_pct = limit_pct;
    s.heartbeat_ns = now;
    s.claim_ns = now;
  }
  unlock(b);
  return got;
}

void board_release(vgpu_board_t* b, int slot) {
  if (!b || slot < 0 || !lock(b)) return;
  advance(b, mono_ns());
  memset(&b->slot[slot], 0, sizeof(b->slot[slot]));
  advance(b, mono_ns());
  unlock(b);
}

void board_heartbeat(vgpu_board_t* b, int slot) {
  if (b && slot >= 0) __atomic_store_n(&b->slot[slot].heartbeat_ns, mono_ns(), __ATOMIC_RELAXED);
}

// Work became outstanding: start accruing fair-share time from now.
void board_enter(vgpu_board_t* b, int slot) {
  if (!b || slot < 0 || !lock(b)) return;
  const uint64_t now = mono_ns();
  advance(b, now);
  vgpu_board_slot_t& s = b->slot[slot];
  s.heartbeat_ns = now;
  s.active = 1;
  s.v_mark = b->v;
  advance(b, now);  // recount with us included
  unlock(b);
}

// Fair-share ns accrued since the last charge; `leave` ends the activity.
uint64_t board_charge(vgpu_board_t* b, int slot, uint64_t wall_ns, bool leave) {
  if (!b || slot < 0 || !lock(b)) return wall_ns;
  const uint64_t now = mono_ns();
  advance(b, now);
  vgpu_board_slot_t& s = b->slot[slot];
  double c = s.active ? b->v - s.v_mark : 0.0;
  if (c < 0) c = 0;
  s.v_mark = b->v;
  s.charged_ns += (uint64_t)c;
  s.busy_ns += wall_ns;
  s.heartbeat_ns = now;
  if (leave) {
    s.active = 0;
    s.running = 0;  // drained: give the running set to a waiter
    advance(b, now);
  }
  unlock(b);
  return (uint64_t)c;
}

// Weighted fair share of `slot` among the slots with work outstanding, counting
// `slot` itself as active: limit_pct(self) / Σ limit_pct(active).  Racy reads
// of other slots are fine: the limiter integrates this over time.
double board_entitlement(vgpu_board_t* b, int slot) {
  if (!b || slot < 0) return 1.0;
  const uint64_t now = mono_ns();
  const double self_w = b->slot[slot].limit_pct > 0 ? b->slot[slot].limit_pct : 1;
  double sum = self_w;
  for (int i = 0; i < VGPU_BOARD_SLOTS; ++i) {
    if (i == slot) continue;
    const vgpu_board_slot_t& s = b->slot[i];
    if (live(s, now)) sum += s.limit_pct > 0 ? s.limit_pct : 1;
  }
  return self_w / sum;
}

namespace {
bool fresh(const vgpu_board_slot_t& s, uint64_t now) {
  return s.pid != 0 && now - s.heartbeat_ns < VGPU_BOARD_STALE_NS;
}
}  // namespace

// The launch admitted by board_gate was not tracked after all (launch error,
// no marker, capture): nothing will drain through board_charge(leave), so
// leave the running set now unless tracked work of ours is still queued.
void board_gate_abort(vgpu_board_t* b, int slot) {
  if (!b || slot < 0 || !lock(b)) return;
  vgpu_board_slot_t& me = b->slot[slot];
  if (!me.active) me.running = 0;
  unlock(b);
}

bool board_gate(vgpu_board_t* b, int slot, int max_running, uint64_t quantum_ns) {
  if (!b || slot < 0 || max_running <= 0 || !lock(b)) return true;
  const uint64_t now = mono_ns();
  vgpu_board_slot_t& me = b->slot[slot];
  me.heartbeat_ns = now;
  // Oldest live waiter other than us (ties: lower slot).
  int oldest = -1;
  int running = 0;
  for (int i = 0; i < VGPU_BOARD_SLOTS; ++i) {
    const vgpu_board_slot_t& s = b->slot[i];
    if (i == slot || !fresh(s, now)) continue;
    running += s.running != 0;
    if (s.wait_since_ns && (oldest < 0 || s.wait_since_ns < b->slot[oldest].wait_since_ns)) oldest = i;
  }
  bool go;
  if (me.running) {
    // Our turn is over and someone waits: stop launching and join the queue.
    // We stay in the running set until our queued work has drained
    // (board_charge(leave) clears `running`), so the waiter never overlaps it.
    go = !(oldest >= 0 && now - me.run_start_ns > quantum_ns);
    if (!go) {
      if (!me.wait_since_ns) me.wait_since_ns = now;
    } else if (me.wait_since_ns) {  // yielded, but nobody waits any more: a new turn
      me.wait_since_ns = 0;
      me.run_start_ns = now;
    }
  } else {
    if (!me.wait_since_ns) me.wait_since_ns = now;
    const bool first = oldest < 0 || me.wait_since_ns < b->slot[oldest].wait_since_ns ||
                       (me.wait_since_ns == b->slot[oldest].wait_since_ns && slot < oldest);
    go = running < max_running && first;
    if (go) {
      me.running = 1;
      me.run_start_ns = now;
      me.wait_since_ns = 0;
    }
  }
  unlock(b);
  return go;
}

// CUs claimed by the other live slots (spatial members of the auto policy).
void board_claims_of_others(vgpu_board_t* b, int slot, uint64_t out[4]) {
  for (int w = 0; w < 4; ++w) out[w] = 0;
  if (!b) return;
  const uint64_t now = mono_ns();
  for (int i = 0; i < VGPU_BOARD_SLOTS; ++i) {
    if (i == slot || !fresh(b->slot[i], now)) continue;
    for (int w = 0; w < 4; ++w) out[w] |= __atomic_load_n(&b->slot[i].cu_claim[w], __ATOMIC_RELAXED);
  }
}

// Claim `n` CUs in whole granules of one CU per XCD (logical bit i -> XCD
// i % num_xcc, cumask.cpp) from `allowed` minus every other live claim; an
// empty `n` releases the claim.  Under the board lock, so two slots never
// claim the same CU.  Returns false when not enough CUs are free.
bool board_claim_cus(vgpu_board_t* b, int slot, uint32_t n, uint32_t num_xcc, const uint64_t allowed[4],
                     uint64_t out[4]) {
  for (int w = 0; w < 4; ++w) out[w] = 0;
  if (!b || slot < 0 || !lock(b)) return false;
  vgpu_board_slot_t& me = b->slot[slot];
  bool ok = true;
  if (n == 0) {
    for (int w = 0; w < 4; ++w) __atomic_store_n(&me.cu_claim[w], 0, __ATOMIC_RELAXED);
  } else {
    uint64_t taken[4] = {};
    const uint64_t now = mono_ns();
    for (int i = 0; i < VGPU_BOARD_SLOTS; ++i) {
      if (i == slot || !fresh(b->slot[i], now)) continue;
      for (int w = 0; w < 4; ++w) taken[w] |= b->slot[i].cu_claim[w];
    }
    const uint32_t g = num_xcc ? num_xcc : 1;  // CUs per granule (one per XCD)
    uint32_t got = 0;
    for (uint32_t base = 0; base + g <= 256 && got < n; base += g) {
      bool free_g = true;
      for (uint32_t k = base; k < base + g && free_g; ++k)
        free_g = (allowed[k / 64] >> (k % 64) & 1) && !(taken[k / 64] >> (k % 64) & 1);
      if (!free_g) continue;
      for (uint32_t k = base; k < base + g; ++k) out[k / 64] |= 1ull << (k % 64);
      got += g;
    }
    ok = got >= n;
    if (!ok)
      for (int w = 0; w < 4; ++w) out[w] = 0;
    for (int w = 0; w < 4; ++w) __atomic_store_n(&me.cu_claim[w], out[w], __ATOMIC_RELAXED);
  }
  unlock(b);
  return ok;
}

// ---- adaptive share policy (auto): a per-GPU A/B, board-coordinated --------------------
void board_auto_join(vgpu_board_t* b, int slot) {
  if (b && slot >= 0) __atomic_store_n(&b->slot[slot].auto_member, 1, __ATOMIC_RELEASE);
}

void board_auto_progress(vgpu_board_t* b, int slot, uint64_t dispatches) {
  if (b && slot >= 0 && dispatches) __atomic_fetch_add(&b->slot[slot].auto_launches, dispatches, __ATOMIC_RELAXED);
}

int board_auto_phase(vgpu_board_t* b) { return b ? __atomic_load_n(&b->auto_phase, __ATOMIC_ACQUIRE) : 0; }

// The lowest live auto member drives the per-GPU state machine:
//   TEMPORAL/SPATIAL (decided) --(>= 2 busy members and a new member count, or
//   `reexplore_ns` since the decision; then, once every member's dispatch rate
//   is steady)--> EXPLORE_T --window--> EXPLORE_S --window--> EXPLORE_T2
//   --window--> SPATIAL if the members' mean dispatch rate on own CUs is at
//   least `min_gain` x their time-shared rate (the mean of the two time-shared
//   windows), else TEMPORAL.
// Steady: each busy member's rate over the last three `bucket_ns` buckets
// varies by at most 30 % -- start-up (graph capture, kernel tuning, the first
// iterations) is not what the pods will run, and an A/B measured there picks
// the wrong mode.  A/B/A: when the two time-shared windows disagree by more
// than 25 % the workload changed under the measurement; the A/B is retried
// (at most three times per member count) and time sharing holds meanwhile.
// Each measurement window opens `settle_ns` after its phase began (masks
// re-applied, queues refilled).  Fewer than two busy members: time sharing (a
// lone pod is not held back there).  A decision is remembered per member
// count: jobs that pause (a step barrier, a checkpoint, a benchmark waiting
// for its peers) return to the decision of their count at once instead of
// re-measuring; an exploration whose member count changes starts over (or
// takes the remembered decision of the new count).  Returns the phase.
int board_auto_lead(vgpu_board_t* b, int slot, uint64_t window_ns, uint64_t settle_ns, uint64_t reexplore_ns,
                    double min_gain, uint64_t bucket_ns, char* note, size_t note_len) {
  if (note && note_len) note[0] = 0;
  if (!b || slot < 0 || !lock(b)) return board_auto_phase(b);
  const uint64_t now = mono_ns();
  int leader = -1, nb = 0;
  int busy[VGPU_BOARD_SLOTS];
  for (int i = 0; i < VGPU_BOARD_SLOTS; ++i) {
    vgpu_board_slot_t& s = b->slot[i];
    if (!fresh(s, now) || !s.auto_member) continue;
    if (leader < 0) leader = i;
    const uint64_t l = __atomic_load_n(&s.auto_launches, __ATOMIC_RELAXED);
    if (l != s.auto_seen) {
      s.auto_seen = l;
      s.auto_busy_ns = now;
    }
    if (now - s.auto_busy_ns < 1000000000ull) busy[nb++] = i;
  }
  int phase = b->auto_phase;
  if (leader != slot) {
    unlock(b);
    return phase;
  }
  // Steadiness buckets: per member, dispatches/s over the last three buckets.
  if (!b->auto_bucket_ns) b->auto_bucket_ns = now;
  if (now - b->auto_bucket_ns >= bucket_ns) {
    const double dt = (now - b->auto_bucket_ns) * 1e-9;
    for (int i = 0; i < VGPU_BOARD_SLOTS; ++i) {
      vgpu_board_slot_t& s = b->slot[i];
      if (!fresh(s, now) || !s.auto_member) continue;
      s.auto_hist[2] = s.auto_hist[1];
      s.auto_hist[1] = s.auto_hist[0];
      s.auto_hist[0] = s.auto_bucket_mark ? (double)(s.auto_seen - s.auto_bucket_mark) / dt : 0.0;
      s.auto_bucket_mark = s.auto_seen ? s.auto_seen : 1;
    }
    b->auto_bucket_ns = now;
  }
  auto steady = [&] {
    for (int k = 0; k < nb; ++k) {
      const double* h = b->slot[busy[k]].auto_hist;
      const double lo = std::min(h[0], std::min(h[1], h[2])), hi = std::max(h[0], std::max(h[1], h[2]));
      if (lo <= 0 || hi > 1.3 * lo) return false;
    }
    return true;
  };
  auto go = [&](int p) {
    __atomic_store_n(&b->auto_phase, p, __ATOMIC_RELEASE);
    b->auto_phase_ns = now;
    b->auto_marked = 0;
    phase = p;
  };
  const bool memo_ok = nb < VGPU_AUTO_MEMO && b->auto_memo_ns[nb] && now - b->auto_memo_ns[nb] < reexplore_ns;
  // A change of the busy-member count counts once it has held for `settle_ns`
  // (pods of one job pause and resume a few ms apart).
  bool count_changed = false;
  if (nb != b->auto_members) {
    if (b->auto_pending_n != nb) {
      b->auto_pending_n = nb;
      b->auto_pending_ns = now;
    }
    count_changed = now - b->auto_pending_ns >= settle_ns;
  } else {
    b->auto_pending_n = -1;
  }
  // A new busy-member count: its remembered decision, else an A/B once steady.
  auto recount = [&] {
    b->auto_members = nb;
    if (memo_ok) {
      go(b->auto_memo_phase[nb]);
      b->auto_want = 0;
      b->auto_score = b->auto_memo_score[nb];
      if (note && note_len)
        snprintf(note, note_len, "%d busy members again: %s (decided %.1f s ago, %.3f x)", nb,
                 phase == VGPU_AUTO_SPATIAL ? "CUs of their own" : "time sharing",
                 (now - b->auto_memo_ns[nb]) * 1e-9, b->auto_memo_score[nb]);
    } else {
      if (phase != VGPU_AUTO_TEMPORAL) go(VGPU_AUTO_TEMPORAL);
      b->auto_want = 3;
    }
  };
  if (phase == VGPU_AUTO_TEMPORAL || phase == VGPU_AUTO_SPATIAL) {
    if (nb < 2) {
      if (phase == VGPU_AUTO_SPATIAL) go(VGPU_AUTO_TEMPORAL);
      b->auto_members = nb;
    } else if (nb != b->auto_members) {
      if (count_changed) recount();
    } else if (b->auto_want > 0) {
      if (steady()) go(VGPU_AUTO_EXPLORE_T);
    } else if (!memo_ok && now - b->auto_phase_ns > reexplore_ns) {
      b->auto_want = 3;
    }
  } else if (nb < 2) {
    go(VGPU_AUTO_TEMPORAL);
    b->auto_members = nb;
  } else if (nb != b->auto_members) {
    if (count_changed) recount();  // the exploration's members changed: its rates would not compare
  } else if (!b->auto_marked) {
    if (now - b->auto_phase_ns >= settle_ns) {
      for (int k = 0; k < nb; ++k) b->slot[busy[k]].auto_mark = b->slot[busy[k]].auto_seen;
      b->auto_phase_ns = now;
      b->auto_marked = 1;
    }
  } else if (now - b->auto_phase_ns >= window_ns) {
    const double secs = (now - b->auto_phase_ns) * 1e-9;
    const int idx = phase == VGPU_AUTO_EXPLORE_T ? 0 : phase == VGPU_AUTO_EXPLORE_S ? 1 : 2;
    for (int k = 0; k < nb; ++k) {
      vgpu_board_slot_t& s = b->slot[busy[k]];
      s.auto_rate[idx] = (double)(s.auto_seen - s.auto_mark) / secs;
    }
    if (phase == VGPU_AUTO_EXPLORE_T) {
      go(VGPU_AUTO_EXPLORE_S);
    } else if (phase == VGPU_AUTO_EXPLORE_S) {
      go(VGPU_AUTO_EXPLORE_T2);
    } else {
      double sum = 0, a0 = 0, a2 = 0;
      int n = 0;
      for (int k = 0; k < nb; ++k) {
        const vgpu_board_slot_t& s = b->slot[busy[k]];
        const double t = 0.5 * (s.auto_rate[0] + s.auto_rate[2]);
        a0 += s.auto_rate[0];
        a2 += s.auto_rate[2];
        if (t > 0) {
          sum += s.auto_rate[1] / t;
          ++n;
        }
      }
      const double score = n ? sum / n : 0.0;
      b->auto_members = nb;
      const bool consistent = a0 > 0 && a2 > 0 && std::max(a0, a2) <= 1.25 * std::min(a0, a2);
      if (!consistent) {
        b->auto_want = b->auto_want > 0 ? b->auto_want - 1 : 0;
        go(VGPU_AUTO_TEMPORAL);
        if (note && note_len)
          snprintf(note, note_len,
                   "%d busy members: time-shared windows disagree (%.0f vs %.0f dispatches/s), %s", nb, a0, a2,
                   b->auto_want ? "measuring again once steady" : "keeping time sharing");
      } else {
        b->auto_score = score;
        b->auto_want = 0;
        go(score >= min_gain ? VGPU_AUTO_SPATIAL : VGPU_AUTO_TEMPORAL);
        if (nb < VGPU_AUTO_MEMO) {
          b->auto_memo_phase[nb] = phase;
          b->auto_memo_ns[nb] = now;
          b->auto_memo_score[nb] = score;
        }
        if (note && note_len)
          snprintf(note, note_len, "%d busy members: own CUs run at %.3f x their time-shared rate -> %s", nb,
                   score, phase == VGPU_AUTO_SPATIAL ? "CUs of their own" : "time sharing");
      }
    }
  }
  unlock(b);
  return phase;
}

int board_running_count(vgpu_board_t* b) {
  if (!b) return 0;
  const uint64_t now = mono_ns();
  int n = 0;
  for (int i = 0; i < VGPU_BOARD_SLOTS; ++i) n += fresh(b->slot[i], now) && b->slot[i].running;
  return n;
}

int board_active_count(vgpu_board_t* b) {
  if (!b) return 0;
  const uint64_t now = mono_ns();
  int n = 0;
  for (int i = 0; i < VGPU_BOARD_SLOTS; ++i) n += live(b->slot[i], now);
  return n;
}

}  // namespace vgpu
