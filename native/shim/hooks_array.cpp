// Cap-refusable array / 3D / mipmapped allocations, code-object (module)
// charging, and IPC pass-through with exporter-only charging.
//
// Reference parity: libvgpu.so hooks
// cuArrayCreate_v2, cuArray3DCreate_v2, cuMipmappedArrayCreate and
// cuModuleLoad*.  It sizes arrays with compute_array_alloc_bytes (420 B) and
// tracks module bytes separately from buffers (allocator.c).  For IPC it
// interposes cuIpcGetMemHandle / cuIpcOpenMemHandle_v2 / cuIpcCloseMemHandle
// (484 B) so RCCL peers do not double-charge shared buffers.
//
// Without these hooks, array and module memory reaches ROCr from inside the
// HIP runtime. The HSA pool interposer charges it but cannot refuse it
// (hooks_hsa.cpp: runtime callers are never refused). A pod could then pass
// its cap through hipMallocArray or hipMalloc3D.  Each allocation path here
// reserves before it allocates, under the InHipAlloc marker, so the pool
// level does not charge the same bytes a second time.
#include <fcntl.h>
#include <sys/stat.h>

#include <algorithm>

#include "common.h"
#include "real.h"
#include "state.h"

using namespace vgpu;

namespace {

struct InHipAlloc {
  InHipAlloc() { ++tl_in_hip_alloc; }
  ~InHipAlloc() { --tl_in_hip_alloc; }
};

inline uint64_t align_up(uint64_t v, uint64_t a) { return (v + a - 1) / a * a; }

// Bytes per element of a driver-API array format x channels.
uint64_t format_bytes(int format, unsigned channels) {
  uint64_t b;
  switch (format) {
    case HIP_AD_FORMAT_UNSIGNED_INT8:
    case HIP_AD_FORMAT_SIGNED_INT8:
      b = 1;
      break;
    case HIP_AD_FORMAT_UNSIGNED_INT16:
    case HIP_AD_FORMAT_SIGNED_INT16:
    case HIP_AD_FORMAT_HALF:
      b = 2;
      break;
    default:  // 32-bit int / float
      b = 4;
  }
  return b * (channels ? channels : 1);
}

uint64_t channel_bytes(const hipChannelFormatDesc* d) {
  if (!d) return 4;
  const int bits = d->x + d->y + d->z + d->w;
  return bits > 0 ? (uint64_t)(bits + 7) / 8 : 1;
}

// Device bytes of a (w x h x d) array of `elem`-byte elements: rows are laid
// out at a 256-byte pitch, as the HIP runtime does for image rows on gfx9.
uint64_t array_bytes(uint64_t elem, uint64_t w, uint64_t h, uint64_t d) {
  return align_up(std::max<uint64_t>(w, 1) * elem, 256) * std::max<uint64_t>(h, 1) * std::max<uint64_t>(d, 1);
}

// A mipmap chain: every level halves each dimension (down to 1).
uint64_t mip_bytes(uint64_t elem, uint64_t w, uint64_t h, uint64_t d, unsigned levels) {
  uint64_t total = 0;
  for (unsigned l = 0; l < std::max(levels, 1u); ++l) {
    total += array_bytes(elem, w, h, d);
    w = std::max<uint64_t>(w / 2, 1);
    if (h) h = std::max<uint64_t>(h / 2, 1);
    if (d) d = std::max<uint64_t>(d / 2, 1);
  }
  return total;
}

// reserve → real allocation → ledger under `key_of()` (or unreserve).
template <class Alloc, class Key>
hipError_t charged(uint64_t bytes, int kind, Alloc&& real_alloc, Key&& key_of) {
  ensure_init();
  State& s = st();
  InHipAlloc in_alloc;
  if (!s.enabled || bytes == 0) return real_alloc();
  suspend_gate();
  const int dev = tl_device;
  charge_context(dev);
  if (!mem_reserve(dev, bytes, kind)) return hipErrorOutOfMemory;
  hipError_t rc = real_alloc();
  if (rc != hipSuccess) {
    mem_unreserve(dev, bytes, kind);
    return rc;
  }
  ledger_add(key_of(), bytes, dev, kind);
  return rc;
}

void uncharge_key(void* key) {
  Alloc a;
  if (key && ledger_take(key, &a)) mem_unreserve(a.dev, a.size, a.kind);
}

// Size of an in-memory code object: an ELF (section headers end the file), or
// an uncompressed clang offload bundle (entries give offset + size).
uint64_t code_object_bytes(const void* image) {
  if (!image) return 0;
  const unsigned char* p = (const unsigned char*)image;
  if (p[0] == 0x7f && p[1] == 'E' && p[2] == 'L' && p[3] == 'F' && p[4] == 2 /* ELFCLASS64 */) {
    uint64_t shoff, phoff;
    uint16_t shentsize, shnum, phentsize, phnum;
    memcpy(&phoff, p + 0x20, 8);
    memcpy(&shoff, p + 0x28, 8);
    memcpy(&phentsize, p + 0x36, 2);
    memcpy(&phnum, p + 0x38, 2);
    memcpy(&shentsize, p + 0x3a, 2);
    memcpy(&shnum, p + 0x3c, 2);
    return std::max<uint64_t>(shoff + (uint64_t)shentsize * shnum, phoff + (uint64_t)phentsize * phnum);
  }
  static const char kBundle[] = "__CLANG_OFFLOAD_BUNDLE__";
  if (!memcmp(p, kBundle, sizeof(kBundle) - 1)) {
    const unsigned char* q = p + sizeof(kBundle) - 1;
    uint64_t n;
    memcpy(&n, q, 8);
    q += 8;
    uint64_t end = 0;
    for (uint64_t i = 0; i < n && i < 4096; ++i) {
      uint64_t off, size, tlen;
      memcpy(&off, q, 8);
      memcpy(&size, q + 8, 8);
      memcpy(&tlen, q + 16, 8);
      q += 24 + tlen;
      end = std::max(end, off + size);
    }
    return end;
  }
  const char* v = env_first("VGPU_MODULE_CHARGE");  // compressed bundles: a flat estimate
  return v ? parse_mem(v) : (1ull << 20);
}

uint64_t file_bytes(const char* fname) {
  struct stat stt;
  return fname && stat(fname, &stt) == 0 ? (uint64_t)stt.st_size : 0;
}

}  // namespace

extern "C" {

// ---- arrays ---------------------------------------------------------------------------
__attribute__((visibility("default"))) hipError_t hipMalloc3D(hipPitchedPtr* pp, hipExtent e) {
  const uint64_t bytes = array_bytes(1, e.width, e.height, e.depth);
  return charged(bytes, kDeviceBuf, [&] { return REAL_HIP(hipMalloc3D)(pp, e); },
                 [&] { return pp->ptr; });
}

__attribute__((visibility("default"))) hipError_t hipMallocArray(hipArray_t* arr, const hipChannelFormatDesc* desc,
                                                                 size_t width, size_t height,
                                                                 unsigned int flags) {
  const uint64_t bytes = array_bytes(channel_bytes(desc), width, height, 1);
  return charged(bytes, kDeviceBuf, [&] { return REAL_HIP(hipMallocArray)(arr, desc, width, height, flags); },
                 [&] { return (void*)*arr; });
}

__attribute__((visibility("default"))) hipError_t hipMalloc3DArray(hipArray_t* arr,
                                                                   const hipChannelFormatDesc* desc,
                                                                   hipExtent e, unsigned int flags) {
  const uint64_t bytes = array_bytes(channel_bytes(desc), e.width, e.height, e.depth);
  return charged(bytes, kDeviceBuf, [&] { return REAL_HIP(hipMalloc3DArray)(arr, desc, e, flags); },
                 [&] { return (void*)*arr; });
}

__attribute__((visibility("default"))) hipError_t hipArrayCreate(hipArray_t* arr, const HIP_ARRAY_DESCRIPTOR* d) {
  const uint64_t bytes = d ? array_bytes(format_bytes(d->Format, d->NumChannels), d->Width, d->Height, 1) : 0;
  return charged(bytes, kDeviceBuf, [&] { return REAL_HIP(hipArrayCreate)(arr, d); },
                 [&] { return (void*)*arr; });
}

__attribute__((visibility("default"))) hipError_t hipArray3DCreate(hipArray_t* arr, const HIP_ARRAY3D_DESCRIPTOR* d) {
  const uint64_t bytes =
      d ? array_bytes(format_bytes(d->Format, d->NumChannels), d->Width, d->Height, d->Depth) : 0;
  return charged(bytes, kDeviceBuf, [&] { return REAL_HIP(hipArray3DCreate)(arr, d); },
                 [&] { return (void*)*arr; });
}

__attribute__((visibility("default"))) hipError_t hipMipmappedArrayCreate(hipMipmappedArray_t* h,
                                                                          HIP_ARRAY3D_DESCRIPTOR* d,
                                                                          unsigned int levels) {
  const uint64_t bytes =
      d ? mip_bytes(format_bytes(d->Format, d->NumChannels), d->Width, d->Height, d->Depth, levels) : 0;
  return charged(bytes, kDeviceBuf, [&] { return REAL_HIP(hipMipmappedArrayCreate)(h, d, levels); },
                 [&] { return (void*)*h; });
}

__attribute__((visibility("default"))) hipError_t hipMallocMipmappedArray(hipMipmappedArray_t* h,
                                                                          const hipChannelFormatDesc* desc,
                                                                          hipExtent e, unsigned int levels,
                                                                          unsigned int flags) {
  const uint64_t bytes = mip_bytes(channel_bytes(desc), e.width, e.height, e.depth, levels);
  return charged(bytes, kDeviceBuf,
                 [&] { return REAL_HIP(hipMallocMipmappedArray)(h, desc, e, levels, flags); },
                 [&] { return (void*)*h; });
}

__attribute__((visibility("default"))) hipError_t hipFreeArray(hipArray_t a) {
  ensure_init();
  uncharge_key((void*)a);
  return REAL_HIP(hipFreeArray)(a);
}

__attribute__((visibility("default"))) hipError_t hipArrayDestroy(hipArray_t a) {
  ensure_init();
  uncharge_key((void*)a);
  return REAL_HIP(hipArrayDestroy)(a);
}

__attribute__((visibility("default"))) hipError_t hipFreeMipmappedArray(hipMipmappedArray_t m) {
  ensure_init();
  uncharge_key((void*)m);
  return REAL_HIP(hipFreeMipmappedArray)(m);
}

__attribute__((visibility("default"))) hipError_t hipMipmappedArrayDestroy(hipMipmappedArray_t m) {
  ensure_init();
  uncharge_key((void*)m);
  return REAL_HIP(hipMipmappedArrayDestroy)(m);
}

// ---- code objects ---------------------------------------------------------------------
__attribute__((visibility("default"))) hipError_t hipModuleLoad(hipModule_t* m, const char* fname) {
  return charged(file_bytes(fname), kModule, [&] { return REAL_HIP(hipModuleLoad)(m, fname); },
                 [&] { return (void*)*m; });
}

__attribute__((visibility("default"))) hipError_t hipModuleLoadData(hipModule_t* m, const void* image) {
  return charged(code_object_bytes(image), kModule, [&] { return REAL_HIP(hipModuleLoadData)(m, image); },
                 [&] { return (void*)*m; });
}

__attribute__((visibility("default"))) hipError_t hipModuleLoadDataEx(hipModule_t* m, const void* image,
                                                                      unsigned int n, hipJitOption* opts,
                                                                      void** vals) {
  return charged(code_object_bytes(image), kModule,
                 [&] { return REAL_HIP(hipModuleLoadDataEx)(m, image, n, opts, vals); },
                 [&] { return (void*)*m; });
}

__attribute__((visibility("default"))) hipError_t hipModuleUnload(hipModule_t m) {
  ensure_init();
  uncharge_key((void*)m);
  return REAL_HIP(hipModuleUnload)(m);
}

// ---- IPC: exporter-only charging --------------------------------------------------------
// The exporting process already holds the charge for the buffer (hipMalloc).
// The importer maps the same HBM, so it records the mapping (kIpcImport,
// charged 0 bytes). A hipFree of an imported pointer then cannot uncharge an
// unrelated buffer, and the monitor can report imported bytes.
// A managed range (virtual device memory under a physical budget) is SVM, not
// a device allocation: the runtime cannot export it.  Say so instead of the
// runtime's bare invalid-value (PyTorch CUDA-IPC tensors / RCCL P2P buffers
// of an oversubscribed pod: docs/config.md, virtual device memory).
// Likewise a VMM-backed range (--suspend-evict: allocations >= 32 MiB are
// hipMemCreate handles mapped at a reserved VA): ROCm's legacy IPC cannot
// export it -- the runtime answers invalid-value, and PyTorch's CUDA-IPC
// sharing then fails in the queue's feeder thread with the consumer waiting
// forever (measured on MI355X, profiles/r6/ipc).  Refuse it up front with the
// remedy instead.
__attribute__((visibility("default"))) hipError_t hipIpcGetMemHandle(hipIpcMemHandle_t* handle, void* dev_ptr) {
  ensure_init();
  if (st().enabled && dev_ptr && vmem_contains(dev_ptr)) {
    VLOG_WARN("hipIpcGetMemHandle(%p): a virtual-device-memory (managed) range cannot be exported over IPC; "
              "set VGPU_VMEM_MANAGED_MIN_MB=-1 for pods that share device buffers between processes",
              dev_ptr);
    return hipErrorNotSupported;
  }
  if (st().enabled && dev_ptr && vmm_owns(dev_ptr)) {
    VLOG_WARN("hipIpcGetMemHandle(%p): a suspend-evict (VMM) range cannot be exported over legacy IPC; "
              "set VGPU_VMEM_MANAGED_MIN_MB=-1 for pods that share device buffers between processes "
              "(their buffers then stay resident across a suspend)",
              dev_ptr);
    return hipErrorNotSupported;
  }
  vmm_ipc_exported(dev_ptr);
  return REAL_HIP(hipIpcGetMemHandle)(handle, dev_ptr);
}

__attribute__((visibility("default"))) hipError_t hipIpcOpenMemHandle(void** dev_ptr, hipIpcMemHandle_t handle,
                                                                      unsigned int flags) {
  ensure_init();
  hipError_t rc = REAL_HIP(hipIpcOpenMemHandle)(dev_ptr, handle, flags);
  if (rc != hipSuccess || !st().enabled || !dev_ptr || !*dev_ptr) return rc;
  size_t size = 0;
  void* base = nullptr;
  if (auto range = REAL_HIP(hipMemGetAddressRange)) (void)range(&base, &size, *dev_ptr);
  ledger_add(*dev_ptr, size, tl_device, kIpcImport);
  ipc_import_account(tl_device, (int64_t)size);
  return rc;
}

__attribute__((visibility("default"))) hipError_t hipIpcCloseMemHandle(void* dev_ptr) {
  ensure_init();
  Alloc a;
  if (dev_ptr && ledger_take_if(dev_ptr, kIpcImport, &a)) ipc_import_account(a.dev, -(int64_t)a.size);
  return REAL_HIP(hipIpcCloseMemHandle)(dev_ptr);
}

}  // extern "C"
