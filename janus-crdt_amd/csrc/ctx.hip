#include <algorithm>
// ctx.hip — context, errors and device buffers of libjanusgpu.
#include <cstring>
#include <vector>

#include "jg_internal.hpp"

namespace jg {

static thread_local char g_err[1024];

void set_error(const char* fmt, ...) {
    va_list ap;
    va_start(ap, fmt);
    std::vsnprintf(g_err, sizeof g_err, fmt, ap);
    va_end(ap);
}

void clear_error() { g_err[0] = 0; }

void fail(int code, const char* fmt, ...) {
    char buf[1024];
    va_list ap;
    va_start(ap, fmt);
    std::vsnprintf(buf, sizeof buf, fmt, ap);
    va_end(ap);
    throw Error{code, buf};
}

void DevBuf::alloc(size_t n) {
    release();
    own = true;
    if (n == 0) return;
    hipError_t e = hipMalloc(&p, n);
    if (e != hipSuccess) {
        p = nullptr;
        (void)hipGetLastError();
        fail(JG_ENOMEM, "hipMalloc(%zu) failed: %s", n, hipGetErrorString(e));
    }
    bytes = n;
}

void DevBuf::release() {
    if (p && own) (void)hipFree(p);
    p = nullptr;
    bytes = 0;
    own = true;
}

void ensure_device(jg_ctx* ctx) { JG_HIP(hipSetDevice(ctx->device)); }

void upload_done(jg_ctx* ctx) {
    JG_HIP(hipEventRecord(ctx->copied, ctx->copy));
    JG_HIP(hipStreamWaitEvent(ctx->stream, ctx->copied, 0));
}

void* scratch(jg_ctx* ctx, DevBuf& b, size_t bytes) {
    if (b.bytes < bytes) {
        JG_HIP(hipStreamSynchronize(ctx->stream));  // the old block may still be in use, also by the digest
        if (ctx->side) JG_HIP(hipStreamSynchronize(ctx->side));      // pipeline's streams (scratch3)
        if (ctx->level1) JG_HIP(hipStreamSynchronize(ctx->level1));
        b.alloc(std::max<size_t>(bytes + bytes / 2, 64 << 10));  // headroom: every growth waits for the streams
    }
    return b.p;
}

}  // namespace jg

extern "C" {

int jg_abi_version(void) { return JG_ABI_VERSION; }

int jg_last_error(char* buf, size_t n) {
    if (!buf || n == 0) return JG_EINVAL;
    std::strncpy(buf, jg::g_err, n - 1);
    buf[n - 1] = 0;
    return JG_OK;
}

int jg_open(int device, jg_ctx** out) {
    return jg::guard([&] {
        JG_REQUIRE(out, JG_EINVAL, "jg_open: out is NULL");
        int count = 0;
        JG_HIP(hipGetDeviceCount(&count));
        JG_REQUIRE(device >= 0 && device < count, JG_EINVAL, "jg_open: device %d of %d", device, count);
        hipDeviceProp_t prop;
        JG_HIP(hipGetDeviceProperties(&prop, device));
        JG_REQUIRE(std::strncmp(prop.gcnArchName, "gfx950", 6) == 0, JG_EINVAL,
                   "jg_open: device %d is %s; this build targets gfx950 only", device, prop.gcnArchName);
        auto* c = new jg_ctx();
        c->device = device;
        c->num_cus = prop.multiProcessorCount;
        try {
            JG_HIP(hipSetDevice(device));
            JG_HIP(hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking));
            JG_HIP(hipStreamCreateWithFlags(&c->copy, hipStreamNonBlocking));
            JG_HIP(hipEventCreateWithFlags(&c->copied, hipEventDisableTiming));
            {  // digest pipeline: chains on the first num_cus/8 CUs, the first level on the others.  The
               // split needs both sets non-empty and the first level the larger one; a small device or
               // partition (a CPX partition has 32 CUs) gets plain streams that share every CU.  CU-masked
               // queues are created blocking (hipStreamDefault) — no library path uses the null stream,
               // so that only orders them against other null-stream work of the process.
                const int chain_cus = c->num_cus / 8;
                const int words = (c->num_cus + 31) / 32;
                bool masked = chain_cus >= 1 && c->num_cus - chain_cus >= 4 * chain_cus;
                if (masked) {
                    std::vector<uint32_t> chain_mask(words, 0), level1_mask(words, 0);
                    for (int cu = 0; cu < c->num_cus; ++cu) (cu < chain_cus ? chain_mask : level1_mask)[cu / 32] |= 1u << (cu % 32);
                    // a queue that refuses a CU mask still runs the pipeline, only with shared SIMDs
                    if (hipExtStreamCreateWithCUMask(&c->side, (uint32_t)words, chain_mask.data()) != hipSuccess ||
                        hipExtStreamCreateWithCUMask(&c->level1, (uint32_t)words, level1_mask.data()) != hipSuccess) {
                        (void)hipGetLastError();
                        if (c->side) (void)hipStreamDestroy(c->side);
                        if (c->level1) (void)hipStreamDestroy(c->level1);
                        c->side = c->level1 = nullptr;
                        masked = false;
                    }
                }
                if (!masked) {
                    JG_HIP(hipStreamCreateWithFlags(&c->side, hipStreamNonBlocking));
                    JG_HIP(hipStreamCreateWithFlags(&c->level1, hipStreamNonBlocking));
                }
                c->cu_masked = masked;
                JG_HIP(hipEventCreateWithFlags(&c->begun, hipEventDisableTiming));
            }
            for (int s = 0; s < 2; ++s) {
                JG_HIP(hipEventCreateWithFlags(&c->level1_done[s], hipEventDisableTiming));
                JG_HIP(hipEventCreateWithFlags(&c->chain_free[s], hipEventDisableTiming));
            }
            c->flags.alloc(256);
            JG_HIP(hipMemset(c->flags.p, 0, 256));
            JG_HIP(hipHostMalloc(&c->hstat, jg::kPinBytes, hipHostMallocDefault));
        } catch (...) {
            delete c;
            throw;
        }
        *out = c;
    });
}

int jg_close(jg_ctx* ctx) {
    return jg::guard([&] {
        if (!ctx) return;
        jg::ensure_device(ctx);
        (void)hipStreamSynchronize(ctx->stream);
        if (ctx->copy) (void)hipStreamSynchronize(ctx->copy);
        if (ctx->side) (void)hipStreamSynchronize(ctx->side);
        if (ctx->level1) (void)hipStreamSynchronize(ctx->level1);
        ctx->scratch.release();
        ctx->scratch2.release();
        ctx->scratch3.release();
        ctx->flags.release();
        if (ctx->hstat) (void)hipHostFree(ctx->hstat);
        (void)hipStreamDestroy(ctx->stream);
        if (ctx->copy) (void)hipStreamDestroy(ctx->copy);
        if (ctx->copied) (void)hipEventDestroy(ctx->copied);
        if (ctx->side) (void)hipStreamDestroy(ctx->side);
        if (ctx->level1) (void)hipStreamDestroy(ctx->level1);
        if (ctx->begun) (void)hipEventDestroy(ctx->begun);
        for (int s = 0; s < 2; ++s) {
            if (ctx->level1_done[s]) (void)hipEventDestroy(ctx->level1_done[s]);
            if (ctx->chain_free[s]) (void)hipEventDestroy(ctx->chain_free[s]);
        }
        delete ctx;
    });
}

int jg_fence(jg_ctx* ctx) {
    return jg::guard([&] {
        auto lk_ = jg::lock(ctx);  // calls on one context are serialised (shared scratch, stream)
        JG_REQUIRE(ctx, JG_EINVAL, "jg_fence: ctx is NULL");
        jg::ensure_device(ctx);
        JG_HIP(hipStreamSynchronize(ctx->stream));
    });
}

int jg_stream(jg_ctx* ctx, void** s) {
    return jg::guard([&] {
        auto lk_ = jg::lock(ctx);  // calls on one context are serialised (shared scratch, stream)
        JG_REQUIRE(ctx && s, JG_EINVAL, "jg_stream: NULL argument");
        *s = (void*)ctx->stream;
    });
}

}  // extern "C"
