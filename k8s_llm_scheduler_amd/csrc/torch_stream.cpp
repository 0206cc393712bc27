// The only translation unit that includes PyTorch headers: it resolves the current PyTorch HIP
// stream so kernels launched from `_C` join PyTorch's stream order and hipGraph captures.
#include <c10/hip/HIPStream.h>

extern "C" void* k8s_current_stream() { return (void*)c10::hip::getCurrentHIPStream().stream(); }
