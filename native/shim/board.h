// Share-board API (board.cpp; layout in include/vgpu/board.h).
#pragma once

#include "vgpu/board.h"

namespace vgpu {

vgpu_board_t* board_map(const char* path);  // create or attach; nullptr on failure
int board_claim(vgpu_board_t* b, int pid, int host_pid, int limit_pct);
void board_release(vgpu_board_t* b, int slot);
void board_heartbeat(vgpu_board_t* b, int slot);
void board_enter(vgpu_board_t* b, int slot);
// Fair-share GPU ns accrued since the previous charge (wall_ns when there is no board).
uint64_t board_charge(vgpu_board_t* b, int slot, uint64_t wall_ns, bool leave);
int board_active_count(vgpu_board_t* b);
// Concurrency gate: true when `slot` may launch now (it is, or just became, one
// of at most `max_running` running slots); false while it must wait.  A runner
// past `quantum_ns` yields to the oldest waiter.
bool board_gate(vgpu_board_t* b, int slot, int max_running, uint64_t quantum_ns);
int board_running_count(vgpu_board_t* b);
void board_gate_abort(vgpu_board_t* b, int slot);  // admitted launch was not tracked
// Adaptive share policy: CU claims of spatial slots.
void board_claims_of_others(vgpu_board_t* b, int slot, uint64_t out[4]);
bool board_claim_cus(vgpu_board_t* b, int slot, uint32_t n, uint32_t num_xcc, const uint64_t allowed[4],
                     uint64_t out[4]);
void board_auto_join(vgpu_board_t* b, int slot);
void board_auto_progress(vgpu_board_t* b, int slot, uint64_t dispatches);
int board_auto_phase(vgpu_board_t* b);
int board_auto_lead(vgpu_board_t* b, int slot, uint64_t window_ns, uint64_t settle_ns, uint64_t reexplore_ns,
                    double min_gain, uint64_t bucket_ns, char* note, size_t note_len);
double board_entitlement(vgpu_board_t* b, int slot);  // weighted fair share among active slots

}  // namespace vgpu
