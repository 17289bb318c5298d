// nm03/cpu_sampler.h — in-process CPU sampling profiler (the reference profiled with
// perf + Hotspot, README.md:92-96, neither of which exists on the GPU boxes).
//
// One POSIX timer on the process's CPU-time clock raises SIGPROF every `period_us` of process CPU
// time; the kernel delivers it to the thread that was running, so samples are proportional to each
// thread's CPU use, kernel time included (a thread inside a system call takes the signal on its way
// back to user space: the sample lands on the libc wrapper — pread64, openat, close — with its
// callers above it). Each sample records the thread id and the interrupted call chain (libgcc
// unwinder through the signal frame). stop() writes the samples, the thread names and the module
// map as text; tools/cpu_profile.py symbolises them offline (llvm-symbolizer) and attributes them.
//
// Off unless started (bench.py --cpu-profile, or NM03_CPU_PROFILE for the CLIs): no handler, no
// timer, no cost.
#pragma once

#include <cstddef>
#include <string>

namespace nm03::prof {

// Starts sampling: one sample per `period_us` of process CPU time, at most `max_samples`, each at
// most `depth` frames deep. False when a sampler is already running or the timer cannot be made.
bool sampler_start(int period_us = 250, size_t max_samples = 1 << 20, int depth = 24);
// Stops the timer and writes every sample to `path` (text, see cpu_sampler.cpp). Returns the
// number of samples written (samples past max_samples are counted as dropped in the file).
size_t sampler_stop(const std::string& path);
bool sampler_running();

}  // namespace nm03::prof
