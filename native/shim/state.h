// Process-global state of the enforcement library.
//
// Reference behaviour (what, not how): lib/nvidia/libvgpu.so keeps a
// per-process view of the shared region, its slot, the allocation chunk list
// (allocator.c: add_chunk/remove_chunk/oom_check), the utilization watcher
// thread and the suspend status.
#pragma once

#include <pthread.h>

#include <atomic>
#include <mutex>
#include <shared_mutex>
#include <unordered_map>
#include <vector>

#include <hip/hip_runtime_api.h>
#include <hsa/hsa.h>

#include "region.h"
#include "vgpu/trace.h"

namespace vgpu {

enum AllocKind : int {
  kDeviceBuf = 0,   // HBM buffer (hipMalloc, hipMallocAsync, hipExtMallocWithFlags, ...)
  kHostSpill = 1,   // oversubscribed allocation backed by pinned host memory
  kManaged = 2,     // hipMallocManaged
  kVmmHandle = 3,   // hipMemCreate physical handle
  kModule = 4,      // code object bytes
  kRuntime = 5,     // HSA pool allocations made outside the HIP hooks (runtime-internal)
  kIpcImport = 6,   // another process's buffer mapped through hipIpcOpenMemHandle (charged 0)
  kPinnedHost = 7,  // page-locked host memory (hipHostMalloc & co.): pinned_host_bytes, not the HBM cap
};

struct Alloc {
  uint64_t size;
  int dev;
  int kind;
};

struct State {
  std::atomic<int> init_done{0};
  bool enabled = false;           // VGPU_DISABLE_CONTROL unset and limits present
  DeviceLimits lim;
  vgpu_shared_region_t* region = nullptr;
  int region_fd = -1;
  int slot = -1;
  int pid = 0;
  bool report_masked_cus = false;
  bool active_oom_killer = false;
  uint64_t context_charge = 0;    // bytes charged per device at first use

  std::mutex ledger_mu;
  std::unordered_map<uintptr_t, Alloc> ledger;

  std::atomic<int> suspended{0};
  // VMM ranges are on the host (vmm.cpp): launches and copies wait like suspended
  std::atomic<int> vmm_evicted{0};
  std::atomic<int64_t> ipc_imported[VGPU_MAX_DEVICES] = {};  // bytes mapped from other processes
  std::atomic<int> dev_touched[VGPU_MAX_DEVICES] = {};
  // Measured runtime memory (mem_sync_runtime): the context charge currently
  // booked per device, and the KFD per-process VRAM counter it is measured from.
  bool ctx_measure = true;        // VGPU_CONTEXT_MEASURE
  uint64_t ctx_max = 0;           // VGPU_CONTEXT_MAX (default 4 GiB)
  std::mutex ctx_mu;
  uint64_t ctx_booked[VGPU_MAX_DEVICES] = {};
  std::atomic<int> kfd_vram_fd[VGPU_MAX_DEVICES];
};

State& st();

// Lazily initialise (pthread_once).  Cheap after the first call.
void ensure_init();

inline vgpu_proc_slot_t* my_slot() {
  State& s = st();
  if (!s.region || s.slot < 0) return nullptr;
  return &s.region->procs[s.slot];
}

// Memory accounting ---------------------------------------------------------
// Reserve `size` bytes of HBM charge on `dev` for this process.  Returns false
// (and counts an OOM event) when the container limit would be exceeded.
bool mem_reserve(int dev, uint64_t size, int kind);
void mem_unreserve(int dev, uint64_t size, int kind);
void ledger_add(void* p, uint64_t size, int dev, int kind);
bool ledger_take(void* p, Alloc* out);
bool ledger_take_if(void* p, int kind, Alloc* out);  // only an entry of that kind
bool app_has_managed();  // the application holds hipMallocManaged memory of its own
// Account without the cap check (runtime-internal memory the application
// cannot be refused): it still counts against the next hipMalloc.
void mem_charge_nofail(int dev, uint64_t size, int kind);
uint64_t mem_limit(int dev);          // 0 = unlimited
void ipc_import_account(int dev, int64_t delta);
uint64_t mem_used(int dev);           // container-wide HBM + host charge
void charge_context(int dev);         // first-touch context charge
// Re-measure the runtime's own VRAM on `dev` (queues and their context-save
// areas, VM-heap slack, code objects ...): KFD's per-process counter minus what
// the ledger already charges becomes the context charge.
void mem_sync_runtime(int dev);
void mem_after_fork();

// Compute limiting ------------------------------------------------------------
void limiter_start();
void limiter_stop();        // exit: stop the limiter thread, release the share board
void limiter_after_fork();
// Called before every dispatch with the number of workgroups it launches;
// blocks while the temporal limiter's bucket is overdrawn.  `fn` = the
// kernel's host stub when known (RCCL kernels are never held, only charged).
// Returns true when the launch must be tracked: call limiter_track after the
// launch on `stream` with its result.  collective: the caller knows the launch
// is a collective's (never held, charged like any launch).  Graphs are held
// before their replay whatever their nodes are (a step boundary).
bool limiter_on_launch(int dev, uint64_t workgroups, const void* fn = nullptr, uint32_t kernels = 1,
                       bool collective = false);
// The kernel whose host stub is `fn` is a collective's (its library is RCCL's,
// or matches VGPU_THROTTLE_EXEMPT).
bool exempt_kernel(const void* fn);
// submit_ns: when the launch was submitted (0 = now); a launch call that may
// return only after its kernel ran (the multi-device launches) passes the time
// before the call, so the marker's interval still covers the kernel.
void limiter_track(int dev, hipStream_t stream, hipError_t launch_rc, uint64_t submit_ns = 0);
void limiter_flush_thread();  // publish this thread's batched slot counters
// Stream captures in progress anywhere in the process: while one is open the
// limiter records and polls markers only on streams that are not capturing (an
// event query on a capturing stream invalidates its capture), and capture
// begin waits for a limiter poll in progress (g_capture_mu).
extern std::atomic<int> g_open_captures;
extern std::shared_mutex g_capture_mu;  // writers: capture begin; readers: limiter-thread markers
void limiter_stats(int dev, uint64_t* charged_ns, uint64_t* busy_ns);
void limiter_share_state(int dev, int64_t out[8]);

// Stream-ordered pools, graph memory and pinned host memory (pools.cpp).
hipError_t pool_alloc_async(void** ptr, size_t size, hipStream_t stream, hipMemPool_t pool,
                            hipError_t (*real)(void**, size_t, hipMemPool_t, hipStream_t, bool));
void pools_sync(bool trim);
void pools_capture_free(const void* ptr);  // hipFreeAsync of a block allocated in a capture
bool pools_any();
void pools_capture_ended(unsigned long long capture_id, hipGraph_t graph);
void pools_graph_instantiated(hipGraph_t graph, hipGraphExec_t exec);
// Explicit graph construction: an alloc node's bytes, a child graph's bytes.
void pools_graph_add_bytes(hipGraph_t graph, uint64_t bytes);
void pools_graph_child(hipGraph_t graph, hipGraph_t child);
void pools_graph_destroyed(const void* graph_or_exec);
uint64_t pools_exec_bytes(hipGraphExec_t exec);
bool pools_graph_admit(hipGraphExec_t exec, int dev, uint64_t* tentative);
void pools_graph_launched(int dev, uint64_t tentative);
bool pinned_reserve(uint64_t size);
void pinned_release(uint64_t size);
void pools_after_fork();

// HSA agents behind HIP device ordinals (cumask.cpp).
bool hsa_gpu_agent(int dev, hsa_agent_t* out);
bool hsa_cpu_agent(hsa_agent_t* out);

// Transparent virtual device memory (vmem.cpp).
bool vmem_enabled();
// Physical HBM (minus a runtime reserve) or the pod's physical budget cannot
// take `size` (already reserved against the cap).
bool vmem_should_spill(int dev, uint64_t size);
// With a physical budget, device allocations of at least VGPU_VMEM_MANAGED_MIN_MB
// are managed ranges from the start (resident while the budget has room).
bool vmem_wants_managed(int dev, uint64_t size);
hipError_t vmem_alloc_managed(void** ptr, size_t size, int dev);
hipError_t vmem_alloc_overflow(void** ptr, size_t size, int dev);
bool vmem_owns(void* p);
// p lies inside a managed range (any offset).
bool vmem_contains(const void* p);
// Async form of vmem_after_copy: the repair runs on the pager thread once the
// operation queued on `stream` has completed.  false: could not queue it.
bool vmem_after_copy_async(const void* dst, const void* src, size_t n, hipStream_t stream);
// Ranges named by an explicitly built graph node (kernel arguments, copy /
// memset pointers) join `key`'s set: a hipGraph_t, or a hipGraphExec_t when exec.
void vmem_graph_note(const void* key, bool exec, void** args, void** extra, const void* const* ptrs, int nptrs);
void vmem_graph_child(hipGraph_t graph, hipGraph_t child);
bool vmem_release(void* p);                 // forget a range before the real free; false if not ours
bool vmem_make_room(int dev, uint64_t need); // demote cold promoted ranges; true if `need` now fits
void vmem_note_plain(int dev);
// Bytes of an application prefetch of [p, p+n) to `dev` (< 0: host) that may run:
// 0 for a range the pager owns, else at most the HBM free beyond the headroom.
size_t vmem_prefetch_allowed(const void* p, size_t n, int dev);
void vmem_budget_books(int dev, uint64_t out[8]);
void vmem_note_use(const void* p, hipStream_t stream);  // a peer copy touches p's range               // a plain buffer was placed: update the plain high-water mark
void vmem_scan_args(void** args, hipStream_t stream);    // HIP-Clang stub argument array
void vmem_scan_extra(void** extra, hipStream_t stream);  // HIP_LAUNCH_PARAM_BUFFER_* kernarg blob
// Graphs: ranges named by captured launches follow capture -> graph -> exec,
// and every launch of the exec stamps them.
unsigned long long vmem_capture_begin_id(hipStream_t stream);  // 0 when not capturing
void vmem_capture_ended(unsigned long long capture_id, hipGraph_t graph);
void vmem_graph_instantiated(hipGraph_t graph, hipGraphExec_t exec);
void vmem_graph_destroyed(const void* graph_or_exec);
void vmem_graph_launched(hipGraphExec_t exec);
uint64_t vmem_graph_ranges(hipGraphExec_t exec);
// A host<->device copy that touched a managed range: KFD moved the pages it
// touched to host memory behind the pager's back; put the resident part back.
bool vmem_copy_touches(const void* dst, const void* src, size_t n);
int vmem_resident_dev(const void* p, size_t n);  // device of a resident managed span in [p, p+n), else -1
void vmem_after_copy(const void* dst, const void* src, size_t n);
void vmem_stats(uint64_t* in_bytes, uint64_t* out_bytes, uint64_t* moves, uint64_t* gpu_bytes, uint64_t* ranges);
void vmem_stop();
void vmem_after_fork();
void suspend_gate();
int cu_count_masked(int dev, int physical);

// CU masks on HSA queues ---------------------------------------------------------
void cumask_on_queue_created(void* agent_handle_ptr, void* queue);
void cumask_on_queue_destroyed(void* queue);
int cumask_reapply_all();

// Event trace (trace.cpp; VGPU_TRACE=<dir>) -----------------------------------------
void trace_open();
void trace_after_fork();
bool trace_on();
void trace_emit(uint32_t type, int dev, uint64_t a, uint64_t b);

extern thread_local int tl_device;

// VMM-backed allocations for suspend with eviction (vmm.cpp) -------------------------
bool vmm_wanted(int dev, uint64_t size);
hipError_t vmm_alloc(void** ptr, size_t size, int dev);
bool vmm_free(void* p);                 // unmap + release + free the VA; false if not ours
bool vmm_owns(const void* p);
int vmm_owner_dev(const void* p);       // device of the range starting at p, -1 if none
void vmm_ipc_exported(const void* p);   // never evict a range another process may map
void vmm_stats(uint64_t out[8]);  // ranges, bytes, evicted bytes, suspend ns, resume ns, cycles, pin ns, map ns
void vmm_after_fork();
void vmem_book_move(int dev, uint64_t bytes, bool to_gpu);
extern std::atomic<int> g_vmm_live;
extern std::atomic<uint64_t> g_hsa_dispatches;        // hooks_hsa.cpp: dispatches through intercept queues
extern std::atomic<int> g_hsa_intercepted_queues;
std::atomic<int>* vmm_hook_enter();
bool vmm_in_scope();  // the calling thread is inside a HookScope past its gate
// Brackets a hook from its gate to the end of its real call while VMM ranges
// exist: the evict thread waits for every open scope before unmapping.
struct HookScope {
  std::atomic<int>* f = nullptr;
  HookScope() {
    if (__builtin_expect(g_vmm_live.load(std::memory_order_relaxed) != 0, 0)) f = vmm_hook_enter();
  }
  ~HookScope() {
    if (f) f->store(0, std::memory_order_release);
  }
  HookScope(const HookScope&) = delete;
  HookScope& operator=(const HookScope&) = delete;
};
// Non-zero while a HIP allocation hook is inside the real runtime call: the
// HSA pool interposer must not charge the same bytes again.
extern thread_local int tl_in_hip_alloc;

// Host-PID resolution (hostpid.cpp) ---------------------------------------------------
const char* kfd_proc_dir();               // VGPU_KFD_PROC_DIR | /sys/class/kfd/kfd/proc
bool pid_ns_is_host();
int hostpid_resolved(int* src);           // KFD-diff result, 0 = none yet
int self_host_pid(int* src);              // best current answer + VGPU_HOSTPID_* source
void hostpid_publish();                   // write it into this process's slot
void hostpid_after_fork();
// Host pids of this container's live processes that are known for sure
// (KFD diff, monitor or host namespace); used to filter smi process lists.
std::vector<int> container_host_pids();

// HSA API table mode (HSA_TOOLS_LIB OnLoad took over the hsa_* hooks).
bool hsa_table_mode();
hsa_status_t real_cu_set_mask(const hsa_queue_t* q, uint32_t bits, const uint32_t* mask);

}  // namespace vgpu
