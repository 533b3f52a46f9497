// resident.cpp — stream-ordered residency of a model's physics image in a device's constant
// segment (the step / env kernels read the image at a fixed address: step.hip, phys<T>()).
//
// One slot per (image kind, device).  The contract of include/pnp.h is that every call is
// asynchronous and stream-ordered, so residency is tracked with events, not host syncs:
//   * a launch that finds its model already resident makes its stream wait on the event recorded
//     after the copy that made it resident (a no-op once that copy has completed), so a launch on
//     stream B never overtakes a copy still queued on stream A;
//   * a launch that needs another model first makes the copying stream wait on the last launch of
//     every stream that has read the old image since it became resident, so a kernel still running
//     on another stream never sees its image overwritten;
//   * the slot mutex is held from the residency check until the launch has been enqueued and its
//     use recorded (ResidentLease), so two host threads cannot interleave check, copy and launch.
// Lock order: a launch that holds two leases (pnp_step: the full image, then the compact or the
// wide image, one at a time) always takes them in the order of ResidentImage.
#include <hip/hip_runtime.h>

#include <mutex>
#include <utility>
#include <vector>

#include "pnp_internal.h"

namespace {

constexpr int kMaxDev = 64;

struct ResidentSlot {
  std::mutex mu;
  const pnp_model* model = nullptr;  // whose image the symbol holds (null: none, or forgotten)
  hipEvent_t copied = nullptr;       // recorded after the last copy into the symbol
  // streams that have launched readers of the current image, with an event recorded after the
  // last such launch on each
  std::vector<std::pair<hipStream_t, hipEvent_t>> users;
};

ResidentSlot g_slots[RES_NKIND][kMaxDev];

int32_t make_event(hipEvent_t* ev) {
  if (*ev) return PNP_OK;
  const hipError_t e = hipEventCreateWithFlags(ev, hipEventDisableTiming);
  if (e != hipSuccess) {
    *ev = nullptr;
    pnp_set_error("resident image: hipEventCreate: %s", hipGetErrorString(e));
    return PNP_ERR_HIP;
  }
  return PNP_OK;
}

}  // namespace

int32_t ResidentLease::acquire(ResidentImage kind, const pnp_model* model, const void* symbol, const void* src,
                               size_t bytes, void* stream) {
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= kMaxDev || kind < 0 || kind >= RES_NKIND) {
    pnp_set_error("resident image: bad device or image kind");
    return PNP_ERR_HIP;
  }
  ResidentSlot& s = g_slots[kind][dev];
  std::unique_lock<std::mutex> lk(s.mu);
  const hipStream_t st = (hipStream_t)stream;
  hipError_t e = hipSuccess;
  if (s.model != model) {
    // the copy waits for every reader of the old image, on whichever stream it was launched
    for (auto& u : s.users)
      if (u.first != st && (e = hipStreamWaitEvent(st, u.second, 0)) != hipSuccess) break;
    if (e == hipSuccess)
      e = hipMemcpyToSymbolAsync(symbol, src, bytes, 0, hipMemcpyDeviceToDevice, st);
    if (e != hipSuccess) {
      pnp_set_error("resident image: %s", hipGetErrorString(e));
      return PNP_ERR_HIP;
    }
    if (const int32_t rc = make_event(&s.copied)) return rc;
    if ((e = hipEventRecord(s.copied, st)) != hipSuccess) {
      s.model = nullptr;  // the copy is queued but cannot be waited on: force a fresh copy next time
      pnp_set_error("resident image: hipEventRecord: %s", hipGetErrorString(e));
      return PNP_ERR_HIP;
    }
    s.model = model;
    // the old readers are ordered before the copy, and the copy before every later reader
    for (auto& u : s.users) (void)hipEventDestroy(u.second);
    s.users.clear();
  } else if ((e = hipStreamWaitEvent(st, s.copied, 0)) != hipSuccess) {
    pnp_set_error("resident image: hipStreamWaitEvent: %s", hipGetErrorString(e));
    return PNP_ERR_HIP;
  }
  slot_ = &s;
  stream_ = stream;
  lock_ = std::move(lk);
  return PNP_OK;
}

int32_t ResidentLease::launched() {
  if (!slot_) return PNP_OK;
  ResidentSlot& s = *static_cast<ResidentSlot*>(slot_);
  const hipStream_t st = (hipStream_t)stream_;
  hipEvent_t* ev = nullptr;
  for (auto& u : s.users)
    if (u.first == st) ev = &u.second;
  if (!ev) {
    s.users.emplace_back(st, nullptr);
    ev = &s.users.back().second;
  }
  int32_t rc = make_event(ev);
  hipError_t e = hipSuccess;
  if (rc == PNP_OK && (e = hipEventRecord(*ev, st)) != hipSuccess) {
    pnp_set_error("resident image: hipEventRecord: %s", hipGetErrorString(e));
    rc = PNP_ERR_HIP;
  }
  // use not recorded: wait for the launch here, so that the next model switch cannot overtake it
  if (rc != PNP_OK) (void)hipStreamSynchronize(st);
  release();
  return rc;
}

void ResidentLease::release() {
  slot_ = nullptr;
  if (lock_.owns_lock()) lock_.unlock();
}

ResidentLease::~ResidentLease() { release(); }

void resident_forget(const pnp_model* model) {
  // a destroyed model is no longer resident anywhere (a new model may reuse its address); its
  // readers stay in the list, so the next copy still waits for them
  for (auto& row : g_slots)
    for (auto& s : row) {
      std::lock_guard<std::mutex> lk(s.mu);
      if (s.model == model) s.model = nullptr;
    }
}
