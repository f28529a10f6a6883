// Resolution of the real HIP / HSA entry points behind our interposers.
//
// The shim never links libamdhip64 / libhsa-runtime64: a PyTorch-ROCm process
// ships its own copies under torch/lib (SONAME libamdhip64.so.7,
// libhsa-runtime64.so.1) and a second runtime in the process would be fatal.
// We look the already-loaded library up by SONAME with RTLD_NOLOAD and only
// fall back to RTLD_NEXT / a plain dlopen for non-PyTorch programs.
#pragma once

#include <dlfcn.h>

#include <hip/hip_runtime_api.h>
#include <hsa/hsa.h>
#include <hsa/hsa_ext_amd.h>

namespace vgpu {

void* hip_lib_handle();
void* hsa_lib_handle();
void* resolve_real(void* handle, const char* name);
// glibc's dlsym (the exported `dlsym` of this library is an interposer, dlsym.cpp).
void* real_dlsym(void* handle, const char* name);
// This library's own definition of a hooked entry point, or nullptr.
void* own_hook(const char* name);
void* amdsmi_lib_handle();
void* recorded_real(const char* name);
bool is_own_address(void* p);
// The real smi entry point for a hook called from `ret_addr` (see real.cpp).
void* smi_real(const char* name, void* ret_addr, void* (*fallback_handle)());
// The caller (a return address) is code of an smi library: libamd_smi calling
// its own or its bundled rocm-smi's entry points through the GOT.  Device-list
// and index virtualisation apply to the application only.
bool called_from_smi_lib(void* ret_addr);
void* rsmi_lib_handle();

}  // namespace vgpu

// Signatures of the HIP entry points we call through (the HIP header adds C++
// template overloads for several of them, so decltype(&fn) is ambiguous).
namespace vgpu {
namespace fnt {
using hipSetDevice = hipError_t (*)(int);
using hipMalloc = hipError_t (*)(void**, size_t);
using hipExtMallocWithFlags = hipError_t (*)(void**, size_t, unsigned int);
using hipMallocAsync = hipError_t (*)(void**, size_t, hipStream_t);
using hipMallocFromPoolAsync = hipError_t (*)(void**, size_t, hipMemPool_t, hipStream_t);
using hipMallocManaged = hipError_t (*)(void**, size_t, unsigned int);
using hipMallocPitch = hipError_t (*)(void**, size_t*, size_t, size_t);
using hipHostMalloc = hipError_t (*)(void**, size_t, unsigned int);
using hipHostFree = hipError_t (*)(void*);
using hipFree = hipError_t (*)(void*);
using hipFreeAsync = hipError_t (*)(void*, hipStream_t);
using hipMemCreate = hipError_t (*)(hipMemGenericAllocationHandle_t*, size_t,
                                    const hipMemAllocationProp*, unsigned long long);
using hipMemRelease = hipError_t (*)(hipMemGenericAllocationHandle_t);
using hipMemAddressReserve = hipError_t (*)(void**, size_t, size_t, void*, unsigned long long);
using hipMemAddressFree = hipError_t (*)(void*, size_t);
using hipMemMap = hipError_t (*)(void*, size_t, size_t, hipMemGenericAllocationHandle_t, unsigned long long);
using hipMemUnmap = hipError_t (*)(void*, size_t);
using hipMemSetAccess = hipError_t (*)(void*, size_t, const hipMemAccessDesc*, size_t);
using hipMemGetAllocationGranularity = hipError_t (*)(size_t*, const hipMemAllocationProp*,
                                                      hipMemAllocationGranularity_flags);
using hipStreamCreateWithFlags = hipError_t (*)(hipStream_t*, unsigned int);
using hipMemGetInfo = hipError_t (*)(size_t*, size_t*);
using hipDeviceTotalMem = hipError_t (*)(size_t*, hipDevice_t);
using hipGetDevicePropertiesR0600 = hipError_t (*)(hipDeviceProp_tR0600*, int);
using hipDeviceGetAttribute = hipError_t (*)(int*, hipDeviceAttribute_t, int);
using hipGetLastError = hipError_t (*)();
using hipStreamSynchronize = hipError_t (*)(hipStream_t);
using hipDeviceSynchronize = hipError_t (*)();
using hipMemcpy = hipError_t (*)(void*, const void*, size_t, hipMemcpyKind);
using hipStreamWaitEvent = hipError_t (*)(hipStream_t, hipEvent_t, unsigned int);
using hipPointerGetAttributes = hipError_t (*)(hipPointerAttribute_t*, const void*);
using hipMemcpyWithStream = hipError_t (*)(void*, const void*, size_t, hipMemcpyKind, hipStream_t);
using hipMemcpyAsync = hipError_t (*)(void*, const void*, size_t, hipMemcpyKind, hipStream_t);
using hipMemcpyHtoD = hipError_t (*)(hipDeviceptr_t, const void*, size_t);
using hipMemcpyDtoH = hipError_t (*)(void*, hipDeviceptr_t, size_t);
using hipMemcpyHtoDAsync = hipError_t (*)(hipDeviceptr_t, const void*, size_t, hipStream_t);
using hipMemcpyDtoHAsync = hipError_t (*)(void*, hipDeviceptr_t, size_t, hipStream_t);
using hipLaunchKernel = hipError_t (*)(const void*, dim3, dim3, void**, size_t, hipStream_t);
using hipExtLaunchKernel = hipError_t (*)(const void*, dim3, dim3, void**, size_t, hipStream_t,
                                          hipEvent_t, hipEvent_t, int);
using hipModuleLaunchKernel = hipError_t (*)(hipFunction_t, unsigned int, unsigned int,
                                             unsigned int, unsigned int, unsigned int,
                                             unsigned int, unsigned int, hipStream_t, void**,
                                             void**);
using hipExtModuleLaunchKernel = hipError_t (*)(hipFunction_t, uint32_t, uint32_t, uint32_t,
                                                uint32_t, uint32_t, uint32_t, size_t,
                                                hipStream_t, void**, void**, hipEvent_t,
                                                hipEvent_t, uint32_t);
using hipLaunchCooperativeKernel = hipError_t (*)(const void*, dim3, dim3, void**, unsigned int,
                                                  hipStream_t);
using hipModuleLaunchCooperativeKernel = hipError_t (*)(hipFunction_t, unsigned int, unsigned int,
                                                        unsigned int, unsigned int, unsigned int,
                                                        unsigned int, unsigned int, hipStream_t,
                                                        void**);
using hipLaunchKernelExC = hipError_t (*)(const hipLaunchConfig_t*, const void*, void**);
using hipGraphLaunch = hipError_t (*)(hipGraphExec_t, hipStream_t);
using hipGraphInstantiate = hipError_t (*)(hipGraphExec_t*, hipGraph_t, hipGraphNode_t*, char*, size_t);
using hipGraphInstantiateWithFlags = hipError_t (*)(hipGraphExec_t*, hipGraph_t, unsigned long long);
using hipGraphInstantiateWithParams = hipError_t (*)(hipGraphExec_t*, hipGraph_t, hipGraphInstantiateParams*);
using hipGraphExecDestroy = hipError_t (*)(hipGraphExec_t);
using hipGraphGetNodes = hipError_t (*)(hipGraph_t, hipGraphNode_t*, size_t*);
using hipGraphNodeGetType = hipError_t (*)(hipGraphNode_t, hipGraphNodeType*);
using hipGraphKernelNodeGetParams = hipError_t (*)(hipGraphNode_t, hipKernelNodeParams*);
using hipGraphChildGraphNodeGetGraph = hipError_t (*)(hipGraphNode_t, hipGraph_t*);
using hipGraphGetEdges = hipError_t (*)(hipGraph_t, hipGraphNode_t*, hipGraphNode_t*, size_t*);
using hipGraphAddDependencies = hipError_t (*)(hipGraph_t, const hipGraphNode_t*, const hipGraphNode_t*, size_t);
using hipGraphRemoveDependencies = hipError_t (*)(hipGraph_t, const hipGraphNode_t*, const hipGraphNode_t*, size_t);
using hipOccupancyMaxActiveBlocksPerMultiprocessor = hipError_t (*)(int*, const void*, int, size_t);
using hipEventCreateWithFlags = hipError_t (*)(hipEvent_t*, unsigned);
using hipEventRecord = hipError_t (*)(hipEvent_t, hipStream_t);
using hipEventQuery = hipError_t (*)(hipEvent_t);
using hipEventDestroy = hipError_t (*)(hipEvent_t);
using hipStreamIsCapturing = hipError_t (*)(hipStream_t, hipStreamCaptureStatus*);
using hipStreamGetDevice = hipError_t (*)(hipStream_t, hipDevice_t*);
using hipStreamDestroy = hipError_t (*)(hipStream_t);
using hipThreadExchangeStreamCaptureMode = hipError_t (*)(hipStreamCaptureMode*);
using hipStreamBeginCapture = hipError_t (*)(hipStream_t, hipStreamCaptureMode);
using hipStreamBeginCaptureToGraph = hipError_t (*)(hipStream_t, hipGraph_t, const hipGraphNode_t*,
                                                    const hipGraphEdgeData*, size_t, hipStreamCaptureMode);
using hipStreamEndCapture = hipError_t (*)(hipStream_t, hipGraph_t*);
using hipStreamGetCaptureInfo = hipError_t (*)(hipStream_t, hipStreamCaptureStatus*, unsigned long long*);
using hipGraphDestroy = hipError_t (*)(hipGraph_t);
using hipGraphClone = hipError_t (*)(hipGraph_t*, hipGraph_t);
using hipGraphAddKernelNode = hipError_t (*)(hipGraphNode_t*, hipGraph_t, const hipGraphNode_t*, size_t,
                                             const hipKernelNodeParams*);
using hipGraphKernelNodeSetParams = hipError_t (*)(hipGraphNode_t, const hipKernelNodeParams*);
using hipGraphExecKernelNodeSetParams = hipError_t (*)(hipGraphExec_t, hipGraphNode_t, const hipKernelNodeParams*);
using hipGraphExecUpdate = hipError_t (*)(hipGraphExec_t, hipGraph_t, hipGraphNode_t*, hipGraphExecUpdateResult*);
using hipGraphAddMemcpyNode = hipError_t (*)(hipGraphNode_t*, hipGraph_t, const hipGraphNode_t*, size_t,
                                             const hipMemcpy3DParms*);
using hipGraphAddMemcpyNode1D = hipError_t (*)(hipGraphNode_t*, hipGraph_t, const hipGraphNode_t*, size_t, void*,
                                               const void*, size_t, hipMemcpyKind);
using hipGraphAddMemsetNode = hipError_t (*)(hipGraphNode_t*, hipGraph_t, const hipGraphNode_t*, size_t,
                                             const hipMemsetParams*);
using hipGraphAddChildGraphNode = hipError_t (*)(hipGraphNode_t*, hipGraph_t, const hipGraphNode_t*, size_t,
                                                 hipGraph_t);
using hipGraphAddMemAllocNode = hipError_t (*)(hipGraphNode_t*, hipGraph_t, const hipGraphNode_t*, size_t,
                                               hipMemAllocNodeParams*);
using hipMemcpy2D = hipError_t (*)(void*, size_t, const void*, size_t, size_t, size_t, hipMemcpyKind);
using hipMemcpy2DAsync = hipError_t (*)(void*, size_t, const void*, size_t, size_t, size_t, hipMemcpyKind,
                                        hipStream_t);
using hipMemcpy3D = hipError_t (*)(const hipMemcpy3DParms*);
using hipMemcpy3DAsync = hipError_t (*)(const hipMemcpy3DParms*, hipStream_t);
using hipMemcpyToSymbol = hipError_t (*)(const void*, const void*, size_t, size_t, hipMemcpyKind);
using hipMemcpyToSymbolAsync = hipError_t (*)(const void*, const void*, size_t, size_t, hipMemcpyKind, hipStream_t);
using hipMemcpyFromSymbol = hipError_t (*)(void*, const void*, size_t, size_t, hipMemcpyKind);
using hipMemcpyFromSymbolAsync = hipError_t (*)(void*, const void*, size_t, size_t, hipMemcpyKind, hipStream_t);
using hipMemset = hipError_t (*)(void*, int, size_t);
using hipMemsetAsync = hipError_t (*)(void*, int, size_t, hipStream_t);
using hipMemsetD8 = hipError_t (*)(hipDeviceptr_t, unsigned char, size_t);
using hipMemsetD8Async = hipError_t (*)(hipDeviceptr_t, unsigned char, size_t, hipStream_t);
using hipMemsetD16 = hipError_t (*)(hipDeviceptr_t, unsigned short, size_t);
using hipMemsetD16Async = hipError_t (*)(hipDeviceptr_t, unsigned short, size_t, hipStream_t);
using hipMemsetD32 = hipError_t (*)(hipDeviceptr_t, int, size_t);
using hipMemsetD32Async = hipError_t (*)(hipDeviceptr_t, int, size_t, hipStream_t);
using hipMemset2D = hipError_t (*)(void*, size_t, int, size_t, size_t);
using hipMemset2DAsync = hipError_t (*)(void*, size_t, int, size_t, size_t, hipStream_t);
using hipMemPoolGetAttribute = hipError_t (*)(hipMemPool_t, hipMemPoolAttr, void*);
using hipMemPoolTrimTo = hipError_t (*)(hipMemPool_t, size_t);
using hipDeviceGetMemPool = hipError_t (*)(hipMemPool_t*, int);
using hipDeviceGetGraphMemAttribute = hipError_t (*)(int, hipGraphMemAttributeType, void*);
using hipDeviceGraphMemTrim = hipError_t (*)(int);
using hipMallocHost = hipError_t (*)(void**, size_t);
using hipHostAlloc = hipError_t (*)(void**, size_t, unsigned int);
using hipFreeHost = hipError_t (*)(void*);
using hipHostRegister = hipError_t (*)(void*, size_t, unsigned int);
using hipHostUnregister = hipError_t (*)(void*);
using hipMalloc3D = hipError_t (*)(hipPitchedPtr*, hipExtent);
using hipMallocArray = hipError_t (*)(hipArray_t*, const hipChannelFormatDesc*, size_t, size_t, unsigned int);
using hipMalloc3DArray = hipError_t (*)(hipArray_t*, const hipChannelFormatDesc*, hipExtent, unsigned int);
using hipArrayCreate = hipError_t (*)(hipArray_t*, const HIP_ARRAY_DESCRIPTOR*);
using hipArray3DCreate = hipError_t (*)(hipArray_t*, const HIP_ARRAY3D_DESCRIPTOR*);
using hipMipmappedArrayCreate = hipError_t (*)(hipMipmappedArray_t*, HIP_ARRAY3D_DESCRIPTOR*, unsigned int);
using hipMallocMipmappedArray = hipError_t (*)(hipMipmappedArray_t*, const hipChannelFormatDesc*, hipExtent,
                                               unsigned int, unsigned int);
using hipFreeArray = hipError_t (*)(hipArray_t);
using hipArrayDestroy = hipError_t (*)(hipArray_t);
using hipFreeMipmappedArray = hipError_t (*)(hipMipmappedArray_t);
using hipMipmappedArrayDestroy = hipError_t (*)(hipMipmappedArray_t);
using hipModuleLoad = hipError_t (*)(hipModule_t*, const char*);
using hipModuleLoadData = hipError_t (*)(hipModule_t*, const void*);
using hipModuleLoadDataEx = hipError_t (*)(hipModule_t*, const void*, unsigned int, hipJitOption*, void**);
using hipModuleUnload = hipError_t (*)(hipModule_t);
using hipIpcGetMemHandle = hipError_t (*)(hipIpcMemHandle_t*, void*);
using hipIpcOpenMemHandle = hipError_t (*)(void**, hipIpcMemHandle_t, unsigned int);
using hipIpcCloseMemHandle = hipError_t (*)(void*);
using hipDeviceGetPCIBusId = hipError_t (*)(char*, int, int);
using hipMemAdvise = hipError_t (*)(const void*, size_t, hipMemoryAdvise, int);
using hipMemPrefetchAsync = hipError_t (*)(const void*, size_t, int, hipStream_t);
using hipMemcpyPeer = hipError_t (*)(void*, int, const void*, int, size_t);
using hipMemcpyPeerAsync = hipError_t (*)(void*, int, const void*, int, size_t, hipStream_t);
using hipMemPrefetchAsync_v2 = hipError_t (*)(const void*, size_t, hipMemLocation, unsigned int, hipStream_t);
using hipMemGetAddressRange = hipError_t (*)(hipDeviceptr_t*, size_t*, hipDeviceptr_t);
using hipGetProcAddress = hipError_t (*)(const char*, void**, int, uint64_t,
                                         hipDriverProcAddressQueryResult*);
using hipMemAllocPitch = hipError_t (*)(hipDeviceptr_t*, size_t*, size_t, size_t, unsigned int);
using hipMemAllocHost = hipError_t (*)(void**, size_t);
using hipLaunchKernel_spt = hipError_t (*)(const void*, dim3, dim3, void**, size_t, hipStream_t);
using hipLaunchCooperativeKernel_spt = hipError_t (*)(const void*, dim3, dim3, void**, uint32_t, hipStream_t);
using hipGraphLaunch_spt = hipError_t (*)(hipGraphExec_t, hipStream_t);
using hipDrvLaunchKernelEx = hipError_t (*)(const HIP_LAUNCH_CONFIG*, hipFunction_t, void**, void**);
using hipHccModuleLaunchKernel = hipError_t (*)(hipFunction_t, uint32_t, uint32_t, uint32_t, uint32_t, uint32_t,
                                                uint32_t, size_t, hipStream_t, void**, void**, hipEvent_t,
                                                hipEvent_t);
using hipExtLaunchMultiKernelMultiDevice = hipError_t (*)(hipLaunchParams*, int, unsigned int);
using hipLaunchCooperativeKernelMultiDevice = hipError_t (*)(hipLaunchParams*, int, unsigned int);
using hipModuleLaunchCooperativeKernelMultiDevice = hipError_t (*)(hipFunctionLaunchParams*, unsigned int,
                                                                   unsigned int);
using hipConfigureCall = hipError_t (*)(dim3, dim3, size_t, hipStream_t);
using hipLaunchByPtr = hipError_t (*)(const void*);
using hipStreamBeginCapture_spt = hipError_t (*)(hipStream_t, hipStreamCaptureMode);
using hipStreamEndCapture_spt = hipError_t (*)(hipStream_t, hipGraph_t*);
using hipMemcpy_spt = hipError_t (*)(void*, const void*, size_t, hipMemcpyKind);
using hipMemcpyAsync_spt = hipError_t (*)(void*, const void*, size_t, hipMemcpyKind, hipStream_t);
using hipMemset_spt = hipError_t (*)(void*, int, size_t);
using hipMemsetAsync_spt = hipError_t (*)(void*, int, size_t, hipStream_t);
using hipMemcpy2D_spt = hipError_t (*)(void*, size_t, const void*, size_t, size_t, size_t, hipMemcpyKind);
using hipMemcpy2DAsync_spt = hipError_t (*)(void*, size_t, const void*, size_t, size_t, size_t, hipMemcpyKind,
                                            hipStream_t);
using hipMemcpy3D_spt = hipError_t (*)(const hipMemcpy3DParms*);
using hipMemcpy3DAsync_spt = hipError_t (*)(const hipMemcpy3DParms*, hipStream_t);
using hipMemset2D_spt = hipError_t (*)(void*, size_t, int, size_t, size_t);
using hipMemset2DAsync_spt = hipError_t (*)(void*, size_t, int, size_t, size_t, hipStream_t);
using hipMemcpyToSymbol_spt = hipError_t (*)(const void*, const void*, size_t, size_t, hipMemcpyKind);
using hipMemcpyToSymbolAsync_spt = hipError_t (*)(const void*, const void*, size_t, size_t, hipMemcpyKind,
                                                  hipStream_t);
using hipMemcpyFromSymbol_spt = hipError_t (*)(void*, const void*, size_t, size_t, hipMemcpyKind);
using hipMemcpyFromSymbolAsync_spt = hipError_t (*)(void*, const void*, size_t, size_t, hipMemcpyKind,
                                                    hipStream_t);
}  // namespace fnt
}  // namespace vgpu

#define VGPU_REAL_IMPL(lib, T, name)                                              \
  ([]() -> T {                                                                    \
    static T p = nullptr;                                                         \
    T v = __atomic_load_n(&p, __ATOMIC_ACQUIRE);                                  \
    if (!v) {                                                                     \
      v = (T)::vgpu::resolve_real(::vgpu::lib(), name);                           \
      __atomic_store_n(&p, v, __ATOMIC_RELEASE);                                  \
    }                                                                             \
    return v;                                                                     \
  }())
// REAL_HIP(hipMalloc)(args...) calls the next definition of hipMalloc.
#define REAL_HIP(fn) VGPU_REAL_IMPL(hip_lib_handle, ::vgpu::fnt::fn, #fn)
// A runtime entry point exported under another (e.g. C++-mangled) name.
#define REAL_HIP_NAMED(T, name) VGPU_REAL_IMPL(hip_lib_handle, T, name)
#define REAL_HSA(fn) VGPU_REAL_IMPL(hsa_lib_handle, decltype(&::fn), #fn)
