// Side streams for off-critical-path work (weight-gradient GEMMs, the x-GEMM beside graph prep).
// fork(main -> side) / join(side -> main) with events; under stream capture both become graph
// edges, so a captured step keeps the concurrency.  Streams and events are created once per device
// (lazily, on the first call, which must not be inside a capture: the library's own warm-up
// happens eagerly in every caller we ship; a first call inside a capture returns an error).
#pragma once

#include <hip/hip_runtime.h>

#include <mutex>

namespace cgr {

struct SideStreams {
  hipStream_t side;
  hipEvent_t ev[16];
  int next;
  // held by cgr_gnn_forward / _backward for their whole enqueue: two host threads driving one
  // device would otherwise re-record each other's ring events between a record and its wait
  std::mutex mu;
  // host-visible error words (ep_bwd.hpp kDevErr*): pinned host memory mapped into the device,
  // written by kernels with plain system-scope stores and read by the host without a sync
  // (cgr_device_errors); null if the pinned allocation failed
  int* err_host;
  int* dev_err;
  // device word written by the fused Adam's step-count kernel: 1 when the error words hold an
  // unpaired-backward timeout (the step's gradients are NaN-poisoned), and k_adam then leaves
  // every parameter and state untouched (optim.hip); null if the allocation failed
  int* adam_gate;
};

// CGR_SINGLE_STREAM=1 in the environment: everything on the caller's stream (A/B of the
// side-stream concurrency against the cross-queue dependency latency it adds in a graph)
bool single_stream();
// CGR_PREP_SPLIT=1 (read per call; tests): the graph bookkeeping always as its own launches
// (graph_prep.hip), never as the x-GEMM's side workgroup (prep_one.hpp)
bool prep_split();

// returns nullptr and sets the library error if the streams cannot be created
SideStreams* side_streams(hipStream_t main);
// the side streams of `device` if they exist (no creation), else nullptr
SideStreams* side_streams_of(int device);

// CGR_UNPAIRED_SPIN_LIMIT (read per call; tests): the unpaired completers' wait bound in polls
// (ep_bwd.hpp); negative = report a timeout at once (exercises the error path)
int unpaired_spin_limit();

// main -> side dependency (side waits for everything enqueued on main so far)
hipError_t fork_to(SideStreams* s, hipStream_t main, hipStream_t side);
// record a point on `from` and make `to` wait for it
hipError_t depend(SideStreams* s, hipStream_t from, hipStream_t to);
// record a point on `from` for a later wait (the ring holds 16 events: wait within 16 records)
hipError_t record_point(SideStreams* s, hipStream_t from, hipEvent_t* ev);

}  // namespace cgr
