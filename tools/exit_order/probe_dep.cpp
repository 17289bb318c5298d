// tools/exit_order: in which order do exit handlers run relative to rocprofv3's tool finalisation?
// This library (a DT_NEEDED dependency of the probe, like libnm03 is of the CLIs) registers a
// handler from its constructor; the probe registers one at the start of main and one after HIP
// has initialised. Each prints a marker; rocprofv3 logs "tool finalization" from its own handler.
#include <cstdio>
#include <cstdlib>

namespace {
void h(int st, void*) { std::fprintf(stderr, "[exit-order] handler registered in a dependency's constructor (status %d)\n", st); }
__attribute__((constructor)) void reg() { on_exit(h, nullptr); }
}  // namespace
