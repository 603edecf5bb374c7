// capi.hip -- error plumbing and ABI version of libuavhip.so (see include/uavhip.h).
#include <cstdarg>
#include <cstdio>
#include <cstring>

#include "common.hpp"

namespace uavhip {
static thread_local char g_err[1024] = "";

void set_error(const char* fmt, ...) {
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(g_err, sizeof g_err, fmt, ap);
    va_end(ap);
}

int check_launch(const char* what) {
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) {
        set_error("%s: %s", what, hipGetErrorString(e));
        return UAVHIP_EHIP;
    }
    return UAVHIP_OK;
}
}  // namespace uavhip

extern "C" const char* uavhip_last_error(void) { return uavhip::g_err; }
extern "C" int32_t uavhip_abi_version(void) { return 5; }

// ------------------------------------------------------------------ the N > 1 trajectory exchange
// Peer-to-peer plumbing for uavhip.dist.IpcAllGather: a rank exports its send buffers
// as IPC handles, every other rank opens them into ITS OWN device's address space (no context on the
// exporter's device) after checking and enabling peer access, and copies out of them on a stream of
// its own device.
// A device's identity across processes: its PCI bus id. Device ordinals are local to a process (a
// rank started with its own HIP_VISIBLE_DEVICES sees its GPU as device 0), so the ranks compare bus
// ids to find a shared device and map a peer's bus id back to THIS process's ordinal before asking
// for peer access (-1: the peer's device is not visible here, so no peer access can be checked).
extern "C" int uavhip_device_pci_id(int32_t device, char* buf, int32_t len) {
    if (!buf || len < 13) {
        uavhip::set_error("uavhip_device_pci_id: buffer of at least 13 bytes required");
        return UAVHIP_EINVAL;
    }
    const hipError_t e = hipDeviceGetPCIBusId(buf, len, device);
    if (e != hipSuccess) {
        uavhip::set_error("uavhip_device_pci_id(%d): %s", device, hipGetErrorString(e));
        return UAVHIP_EHIP;
    }
    return UAVHIP_OK;
}

extern "C" int uavhip_device_from_pci_id(const char* pci_id, int32_t* device) {
    if (!pci_id || !device) {
        uavhip::set_error("uavhip_device_from_pci_id: NULL pointer");
        return UAVHIP_EINVAL;
    }
    int d = -1;
    if (hipDeviceGetByPCIBusId(&d, pci_id) != hipSuccess) {
        (void)hipGetLastError();
        d = -1;
    }
    *device = d;
    return UAVHIP_OK;
}

extern "C" int uavhip_peer_access(int32_t peer_device, int32_t* can_access) {
    int cur = 0, can = 0;
    if (!can_access) {
        uavhip::set_error("uavhip_peer_access: NULL pointer");
        return UAVHIP_EINVAL;
    }
    *can_access = 0;
    if (hipGetDevice(&cur) != hipSuccess) {
        uavhip::set_error("uavhip_peer_access: hipGetDevice failed");
        return UAVHIP_EHIP;
    }
    if (peer_device == cur) {  // the same device (several ranks on one GPU): no peer mapping needed
        *can_access = 1;
        return UAVHIP_OK;
    }
    if (hipDeviceCanAccessPeer(&can, cur, peer_device) != hipSuccess) {
        uavhip::set_error("uavhip_peer_access: hipDeviceCanAccessPeer(%d, %d) failed", cur, peer_device);
        return UAVHIP_EHIP;
    }
    if (!can) return UAVHIP_OK;
    const hipError_t e = hipDeviceEnablePeerAccess(peer_device, 0);
    if (e != hipSuccess && e != hipErrorPeerAccessAlreadyEnabled) {
        (void)hipGetLastError();
        uavhip::set_error("uavhip_peer_access: hipDeviceEnablePeerAccess(%d) from %d: %s", peer_device, cur,
                          hipGetErrorString(e));
        return UAVHIP_EHIP;
    }
    (void)hipGetLastError();  // clear an already-enabled status
    *can_access = 1;
    return UAVHIP_OK;
}

extern "C" int uavhip_ipc_export(const void* ptr, void* handle, uint64_t* offset) {
    if (!ptr || !handle || !offset) {
        uavhip::set_error("uavhip_ipc_export: NULL pointer");
        return UAVHIP_EINVAL;
    }
    hipDeviceptr_t base = nullptr;
    size_t size = 0;
    if (hipMemGetAddressRange(&base, &size, (hipDeviceptr_t)ptr) != hipSuccess) {
        uavhip::set_error("uavhip_ipc_export: hipMemGetAddressRange failed");
        return UAVHIP_EHIP;
    }
    hipIpcMemHandle_t h;
    const hipError_t e = hipIpcGetMemHandle(&h, (void*)base);
    if (e != hipSuccess) {
        uavhip::set_error("uavhip_ipc_export: hipIpcGetMemHandle: %s", hipGetErrorString(e));
        return UAVHIP_EHIP;
    }
    static_assert(sizeof(h) == UAVHIP_IPC_HANDLE_BYTES, "IPC handle size");
    memcpy(handle, &h, sizeof h);
    *offset = (uint64_t)((const char*)ptr - (const char*)base);
    return UAVHIP_OK;
}

extern "C" int uavhip_ipc_open(const void* handle, uint64_t offset, void** ptr) {
    if (!handle || !ptr) {
        uavhip::set_error("uavhip_ipc_open: NULL pointer");
        return UAVHIP_EINVAL;
    }
    hipIpcMemHandle_t h;
    memcpy(&h, handle, sizeof h);
    void* base = nullptr;
    const hipError_t e = hipIpcOpenMemHandle(&base, h, hipIpcMemLazyEnablePeerAccess);
    if (e != hipSuccess) {
        uavhip::set_error("uavhip_ipc_open: hipIpcOpenMemHandle: %s", hipGetErrorString(e));
        return UAVHIP_EHIP;
    }
    *ptr = (char*)base + offset;
    return UAVHIP_OK;
}

extern "C" int uavhip_ipc_close(void* base) {
    if (hipIpcCloseMemHandle(base) != hipSuccess) {
        uavhip::set_error("uavhip_ipc_close: hipIpcCloseMemHandle failed");
        return UAVHIP_EHIP;
    }
    return UAVHIP_OK;
}

extern "C" int uavhip_copy_async(void* dst, const void* src, uint64_t bytes, uavhip_stream_t stream) {
    if ((!dst || !src) && bytes) {
        uavhip::set_error("uavhip_copy_async: NULL pointer");
        return UAVHIP_EINVAL;
    }
    const hipError_t e = hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToDevice, (hipStream_t)stream);
    if (e != hipSuccess) {
        uavhip::set_error("uavhip_copy_async: %s", hipGetErrorString(e));
        return UAVHIP_EHIP;
    }
    return UAVHIP_OK;
}
