// jit.cpp — run-time compiled bit-sliced kernels for wide byte-wise codes
// (more than 4 outputs: m > 4 encodes and updates, decodes of > 4 erasures).
//
// Each distinct coefficient matrix gets its own straight-line kernel
// (bitslice.cpp: 8 x 8 bit transposes and a four-Russians XOR program with
// the matrix baked in as constants), compiled with hiprtc for gfx950 and
// loaded as a module on the context's device.  Compilation takes ~1 s, so by
// default it runs on a background thread (MEC_BITSLICE=1) while the matrix's
// calls keep running on gf8_mg_kernel; once the module is loaded every later
// call with that matrix launches it.  MEC_BITSLICE=2 compiles on the calling
// thread at first use (benchmarks, tests), 0 never uses it.  At most
// MEC_JIT_MAX_KERNELS (default 512) matrices per context are compiled, and
// at most MEC_JIT_MAX_QUEUED (16) wait in the compile queue at once (a decode
// workload walking many erasure patterns queues no more than that; a
// pattern past it is queued on a later call); beyond either the one-pass
// kernel serves the call.  mec_destroy cancels the context's queued
// compiles, waits only for one already running and for the last launch of
// each of its kernels on each stream, then unloads the modules.
#include <hip/hiprtc.h>

#include <chrono>
#include <condition_variable>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <algorithm>
#include <deque>
#include <thread>

#include "bitslice.hpp"
#include "ctx.hpp"
#include "knobs.hpp"
#include "launch_plan.hpp"

namespace mec {
namespace core {
namespace {

// One background compiler thread per process, FIFO.
struct Worker {
    std::mutex mu;
    std::condition_variable cv;
    std::deque<std::function<void()>> jobs;
    bool started = false;
    void post(std::function<void()> f) {
        std::lock_guard<std::mutex> g(mu);
        jobs.push_back(std::move(f));
        if (!started) {
            started = true;
            std::thread([this] {
                for (;;) {
                    std::function<void()> f;
                    {
                        std::unique_lock<std::mutex> lk(mu);
                        cv.wait(lk, [&] { return !jobs.empty(); });
                        f = std::move(jobs.front());
                        jobs.pop_front();
                    }
                    f();
                }
            }).detach();
        }
        cv.notify_one();
    }
};
Worker &worker() {
    static Worker *w = new Worker;  // never destroyed: the detached thread may outlive static destruction
    return *w;
}

// hiprtc source -> code object for the device's arch -> module on `device`.
void compile(JitKernel &k, const std::string &src, int device, const std::string &arch) {
    const auto t0 = std::chrono::steady_clock::now();
    hiprtcProgram prog = nullptr;
    std::string err;
    std::vector<char> code;
    if (hiprtcCreateProgram(&prog, src.c_str(), "mec_bs.hip", 0, nullptr, nullptr) != HIPRTC_SUCCESS) {
        err = "hiprtcCreateProgram";
    } else {
        const std::string a = "--offload-arch=" + arch;
        const char *opts[] = {a.c_str(), "-O3", "-std=c++17"};
        const hiprtcResult r = hiprtcCompileProgram(prog, 3, opts);
        if (r != HIPRTC_SUCCESS) {
            size_t n = 0;
            hiprtcGetProgramLogSize(prog, &n);
            std::string log(n, '\0');
            if (n) hiprtcGetProgramLog(prog, &log[0]);
            err = std::string("hiprtc: ") + hiprtcGetErrorString(r) + ": " + log.substr(0, 400);
        } else {
            size_t n = 0;
            hiprtcGetCodeSize(prog, &n);
            code.resize(n);
            hiprtcGetCode(prog, code.data());
        }
        hiprtcDestroyProgram(&prog);
    }
    if (err.empty()) {
        DeviceGuard dg(device);
        hipError_t e = hipModuleLoadData(&k.mod, code.data());
        if (e == hipSuccess) e = hipModuleGetFunction(&k.fn, k.mod, "mec_bs");
        if (e != hipSuccess) err = std::string("module: ") + hipGetErrorString(e);
    }
    k.compile_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    k.err = err;
    k.state.store(err.empty() ? 1 : -1, std::memory_order_release);
    if (!err.empty()) std::fprintf(stderr, "libmec: bit-sliced kernel not built (%s); gf8_mg_kernel serves it\n", err.c_str());
}

uint64_t env_u64(const char *name, uint64_t dflt) {
    const char *e = std::getenv(name);
    return e && *e ? std::strtoull(e, nullptr, 10) : dflt;
}

}  // namespace

// Which wide launches take the bit-sliced kernel (MEC_BITSLICE unset, 1 or
// 2): every byte-wise launch of more than 4 outputs on chunks that are a
// multiple of 16 bytes.  With the wave caps of plan_bs it leads the
// one-pass kernel on every wide shape measured, the Vandermonde encodes
// under 12 sources included (RS(10,6)@256 KiB encode 78.9-79.9 % against
// 74.7-77.7, RS(8,5)@16 KiB 82.8-83.4 against 76.3-80.1, RS(4,12)@1 MiB
// 81.8 against 77.7-78.8; ISA-L Cauchy(4,12) ties, 75-76 both), and by
// 7-24 points on the rest (tools/wide_ab.py, profiles/r05/wide_*.jsonl).
// The one-pass kernel serves the rest: a matrix whose kernel is still
// compiling, other chunk sizes, MEC_BITSLICE=0.  MEC_BITSLICE=3 also
// compiles synchronously, like 2 (A/B).
bool jit_wanted(const mec_ctx *c, size_t nd, size_t ns, const Mat &coef, bool gathered) {
    (void)ns;
    (void)coef;
    (void)gathered;
    const int64_t kn = detail::knob(detail::kKnobBitslice);
    return kn != 0 && c->byte_wise() && nd > size_t(kMaxRows) && c->cs % 16 == 0;
}

// Row 0 and column 0 all ones: a Vandermonde-structured encode (Jerasure's
// distribution rows, ISA-L gf_gen_rs_matrix), which takes its own wave cap.
bool coef_vand(const Mat &coef, size_t nd, size_t ns) {
    bool vand = true;
    for (size_t j = 0; j < ns && vand; ++j) vand = coef[j] == 1;
    for (size_t r = 0; r < nd && vand; ++r) vand = coef[r * ns] == 1;
    return vand;
}

// The kernel for (coef, accumulate, addressing), compiling it if needed;
// nullptr while it compiles (async), past the cap, or after a failure.
JitKernel *jit_kernel(mec_ctx *c, const Mat &coef, size_t nd, size_t ns, bool accumulate, bool gather, bool twin) {
    std::string key(reinterpret_cast<const char *>(coef.data()), nd * ns);
    key += char(nd);
    key += char(ns);
    key += char(accumulate ? 1 : 0);
    key += char(gather ? 1 : 0);
    const int64_t wk = detail::knob(detail::kKnobBsWaves);  // experiments (mec_set_knob)
    const int waves = wk == detail::kKnobUnset ? 0 : int(wk);
    key += char(waves);
    // gathered: one straight-line tile per block (the strided kernel's
    // shape), unless MEC_BS_TPB asks for a loop over several tiles per
    // pointer-row read.  Every form keeps 4 sources' loads ahead of the
    // combine: RS(16,8) strided 141 VGPRs (163 with every load first),
    // gathered 156 (207), looped 165 (235) — 3 waves per SIMD, no scratch
    // (test_abi.py::test_bitslice_kernels_compile_for_gfx950).
    const uint32_t tpb = gather ? std::min<uint32_t>(detail::bs_gather_tpb(), 255u) : 1u;
    const bool loop = tpb > 1;
    key += char(tpb);
    const int64_t pk = detail::knob(detail::kKnobBsPrefetch);
    const int prefetch = pk == detail::kKnobUnset ? 4 : int(pk);
    key += char(prefetch);
    // scheduling fences between sources (bitslice.hpp): one source's
    // combinations live at a time.  Gathered kernels take them — RS(16,8)
    // 167 -> 127 VGPRs, 3 -> 4 waves per SIMD, one-map batches +2-5 points;
    // strided ones do not — 141 -> 127 VGPRs there loses 1-4 points on the
    // encodes (more waves only lengthen the memory queue;
    // profiles/r05/wide_fence_twin_box7.jsonl)
    const int64_t fk = detail::knob(detail::kKnobBsFence);
    const bool fence = fk == detail::kKnobUnset ? gather : fk != 0;
    key += char(fence ? 1 : 0);
    key += char(twin ? 1 : 0);
    // gathered: the pointer row in one vector load (bitslice.hpp vrow)
    const int64_t vk = detail::knob(detail::kKnobBsVrow);
    const bool vrow = vk == detail::kKnobUnset || vk != 0;
    key += char(vrow ? 1 : 0);
    JitCache &J = c->jit;
    const bool sync = detail::knob(detail::kKnobBitslice) >= 2;
    const std::shared_ptr<JitShared> sh = J.sh;
    std::shared_ptr<JitKernel> k;
    bool fresh = false;
    {
        std::unique_lock<std::mutex> g(J.mu);
        auto it = J.map.find(key);
        if (it != J.map.end()) {
            k = it->second;
        } else {
            if (J.map.size() >= J.cap) return nullptr;
            {
                std::lock_guard<std::mutex> q(sh->mu);
                // async: bound the compiles this context has waiting (the
                // pattern is tried again on a later call)
                if (!sync && sh->pending >= J.max_queued) return nullptr;
                ++sh->pending;
            }
            k = std::make_shared<JitKernel>();
            k->tpb = tpb;
            J.map.emplace(key, k);
            fresh = true;
        }
    }
    if (fresh) {
        auto src = std::make_shared<std::string>(bs_source(twin ? bs_build_twin(int(nd), int(ns), accumulate) : bs_build(coef.data(), int(nd), int(ns), accumulate),
                      gather, waves, prefetch, loop, fence, vrow));
        const int device = c->device;
        const std::string arch = J.arch;
        // a job runs unless its context was released meanwhile; it holds
        // the shared state and the kernel, never the context
        auto job = [k, src, device, arch, sh] {
            {
                std::lock_guard<std::mutex> g(sh->mu);
                if (sh->cancelled) {
                    --sh->pending;
                    k->err = "context released before the compile ran";
                    k->state.store(-1, std::memory_order_release);
                    sh->cv.notify_all();
                    return;
                }
                ++sh->running;
            }
            compile(*k, *src, device, arch);
            std::lock_guard<std::mutex> g(sh->mu);
            --sh->running;
            --sh->pending;
            sh->compile_ms += k->compile_ms;
            if (k->state.load() > 0) ++sh->ready;
            else ++sh->failed;
            sh->cv.notify_all();
        };
        if (sync) job();
        else worker().post(job);
    }
    if (sync && k->state.load(std::memory_order_acquire) == 0) {  // another thread compiling it: wait
        std::unique_lock<std::mutex> g(sh->mu);
        sh->cv.wait(g, [&] { return k->state.load(std::memory_order_acquire) != 0; });
    }
    return k->state.load(std::memory_order_acquire) > 0 ? k.get() : nullptr;
}

int jit_launch(mec_ctx *c, JitKernel *k, const BsLaunch &L0, hipStream_t stream) {
    BsLaunch L = L0;
    L.tpb = L.stab ? k->tpb : 1u;  // the tiles per block this kernel was built for
    BsParams p{};
    p.src = L.src;
    p.dst = L.dst;
    p.sss = L.src_stripe_stride;
    p.dss = L.dst_stripe_stride;
    p.stab = L.stab;
    p.dtab = L.dtab;
    p.sstride = L.sstride;
    p.dstride = L.dstride;
    p.chunk = uint32_t(L.len);
    for (int j = 0; j < L.k; ++j) p.src_off[j] = L.src_off[j];
    for (int r = 0; r < L.rows; ++r) p.dst_off[r] = L.dst_off[r];
    for (uint32_t s0 = 0; s0 < L.n_stripes;) {
        const detail::KernelPlan pl = detail::plan_bs(L, s0);
        if (!pl.ok) return fail(MEC_EINVAL, "bit-sliced launch: %s", pl.why);
        p.tiles = pl.geo.tiles;
        p.tpb = pl.tpb;
        p.xcd = pl.xcd;
        p.win = pl.win;
        p.s0 = s0;
        if (!L.stab) {
            p.src = L.src + int64_t(s0) * L.src_stripe_stride;
            p.dst = L.dst + int64_t(s0) * L.dst_stripe_stride;
        }
        size_t sz = sizeof(p);
        void *cfg[] = {HIP_LAUNCH_PARAM_BUFFER_POINTER, &p, HIP_LAUNCH_PARAM_BUFFER_SIZE, &sz, HIP_LAUNCH_PARAM_END};
        HIP_TRY(hipModuleLaunchKernel(k->fn, uint32_t(pl.grid), 1, 1, pl.bt, 1, 1, pl.lds_dynamic, stream, nullptr, cfg));
        s0 += pl.ns;
    }
    {  // the module's last launch on this stream (jit_release waits for it)
        std::lock_guard<std::mutex> g(k->ev_mu);
        hipEvent_t ev = nullptr;
        for (auto &pr : k->ev)
            if (pr.first == stream) ev = pr.second;
        if (!ev) {
            HIP_TRY(hipEventCreateWithFlags(&ev, hipEventDisableTiming | hipEventReleaseToDevice));
            k->ev.emplace_back(stream, ev);
        }
        HIP_TRY(hipEventRecord(ev, stream));
    }
    c->jit.launches.fetch_add(1, std::memory_order_relaxed);
    return MEC_OK;
}

void jit_init(mec_ctx *c) {
    c->jit.cap = size_t(env_u64("MEC_JIT_MAX_KERNELS", 512));
    c->jit.max_queued = uint32_t(std::max<uint64_t>(1, env_u64("MEC_JIT_MAX_QUEUED", 16)));
}

// no device-wide synchronize (it waited on every stream of the
// device, other contexts' resident queue grids and a hung one included):
// queued compiles are cancelled, a running one is waited for, and each
// module is unloaded after the last launch it made on each stream.
void jit_release(mec_ctx *c) {
    JitCache &J = c->jit;
    {
        std::unique_lock<std::mutex> g(J.sh->mu);
        J.sh->cancelled = true;
        J.sh->cv.wait(g, [&] { return J.sh->running == 0; });
    }
    DeviceGuard dg(c->device);
    for (auto &kv : J.map) {
        JitKernel &k = *kv.second;
        std::lock_guard<std::mutex> g(k.ev_mu);
        for (auto &pr : k.ev) {
            (void)hipEventSynchronize(pr.second);
            (void)hipEventDestroy(pr.second);
        }
        k.ev.clear();
        if (k.mod) (void)hipModuleUnload(k.mod);
        k.mod = nullptr;
        k.fn = nullptr;
    }
    J.map.clear();
}

}  // namespace core
}  // namespace mec
