// fork_guard.h — the boundary's fork-after-initialisation check.
//
// The reference's callers fork: StandardNLSFitter._fit_parallel and Experiment.run start
// multiprocessing Pools (fitters.py:421-423, experiments.py:381-384). A child forked
// BEFORE the parent's first GPU call initialises HIP itself and works (include/dfmi.h).
// A child forked AFTER it inherits a copy of the parent's HIP runtime state (queues,
// doorbells, device mappings) that no longer belongs to it: any HIP call there is
// undefined behaviour. libdfmi.so records the pid of the process that initialised HIP
// and refuses, before any runtime call, every entry point called from another pid.
#pragma once
#include <string>

// Empty when the calling process `cur_pid` may use the HIP state initialised by
// `init_pid` (0: not initialised yet); otherwise the error message naming both pids.
inline std::string dfmi_fork_guard(long init_pid, long cur_pid) {
  if (init_pid == 0 || init_pid == cur_pid) return std::string();
  return "libdfmi.so was initialised on the GPU in process " + std::to_string(init_pid) +
         "; this process (" + std::to_string(cur_pid) +
         ") is a fork of it and inherits that HIP state, which it cannot use: fork before the "
         "first GPU call (the Pool pattern of fitters.py:421-423), or use the 'spawn' start method";
}
