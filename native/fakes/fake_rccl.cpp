// A stand-in for librccl's kernel host stubs (CPU tests): the enforcement
// library exempts kernels whose host stub lives in an rccl/nccl library from
// the temporal limiter (native/shim/limiter.cpp, exempt_kernel).
extern "C" __attribute__((visibility("default"))) void rccl_fake_kernel_stub() {}
