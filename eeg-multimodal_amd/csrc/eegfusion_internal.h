// eegfusion_internal.h — enums shared by the kernels and the C-ABI (mirrors include/eegfusion.h).
#pragma once
#include "../../include/eegfusion.h"

extern int g_ln_rpw;  // layernorm.hip: rows per wave of eegf_ln_fwd (eegf_tune key 6)
extern int g_ln_bwd_rpb;  // layernorm.hip: rows per workgroup of eegf_ln_bwd at rows >= 65536 (eegf_tune key 7)

// Launch log (diagnostics; eegf_launch_log_read / _reset in launch_log.hip): every kernel launch of
// the library goes through EEGF_LAUNCH, which counts it per kernel (its host stub address, i.e. one
// entry per template instantiation) before hipLaunchKernelGGL.  Host-side only: a mutex and a map
// update per launch, nothing on the device.
void eegf_note_launch(const void* kernel);
#define EEGF_LAUNCH(kernel, ...)                                   \
  do {                                                             \
    eegf_note_launch(reinterpret_cast<const void*>(kernel));       \
    hipLaunchKernelGGL(kernel, __VA_ARGS__);                       \
  } while (0)
