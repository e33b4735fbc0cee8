// mh_comm.cpp — RCCL communicators of the C ABI (include/mitsuba_hip.h,
// "Multi-GPU").  Host code only.
//
// The reference has no collective at all: each process renders on one device
// (src/render/integrator.cpp:276-390) and Dr.Jit's AD stays on that device.
// The sample-slab split of SURVEY.md §8(e) needs exactly one kind of exchange,
// a float sum (film, W image, gradients), so this layer is that sum over RCCL
// (xGMI within a node) and nothing else.
//
// RCCL is bound on first use with dlopen + dlsym instead of a link-time
// dependency: the library then loads on hosts without RCCL (the comm entry
// points report MH_ERR_UNSUPPORTED there), and a process that already mapped
// another RCCL (torch's bundled librccl.so carries no SONAME) keeps its own.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>  // types and signatures only; the entry points come from dlsym

#include <dlfcn.h>

#include <chrono>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <thread>
#include <string>
#include <vector>

#include "mh_internal.hpp"
#include "../../include/mitsuba_hip.h"

struct mh_comm {
    ncclComm_t comm = nullptr;
    int nranks = 0, rank = 0, device = 0;
    int users = 0;         // scenes this communicator is attached to (mh_scene_set_comm)
    bool aborted = false;  // aborted after a failure: every later collective fails fast
};

namespace {

struct Rccl {
    bool ok = false;
    std::string why;
    decltype(&ncclGetUniqueId) get_unique_id = nullptr;
    decltype(&ncclCommInitRank) init_rank = nullptr;
    decltype(&ncclCommInitAll) init_all = nullptr;
    decltype(&ncclCommDestroy) destroy = nullptr;
    decltype(&ncclAllReduce) all_reduce = nullptr;
    decltype(&ncclReduce) reduce = nullptr;
    decltype(&ncclGroupStart) group_start = nullptr;
    decltype(&ncclGroupEnd) group_end = nullptr;
    decltype(&ncclGetErrorString) error_string = nullptr;
    decltype(&ncclCommGetAsyncError) async_error = nullptr;
    decltype(&ncclCommAbort) abort = nullptr;
};

Rccl &rccl() {
    static Rccl R;
    static std::once_flag once;
    std::call_once(once, [] {
        void *h = nullptr;
        for (const char *name : {"librccl.so.1", "/opt/rocm/lib/librccl.so.1", "librccl.so"})
            if ((h = dlopen(name, RTLD_NOW | RTLD_LOCAL))) break;
        if (!h) {
            const char *e = dlerror();
            R.why = std::string("RCCL (librccl.so.1) could not be loaded: ") + (e ? e : "not found");
            return;
        }
        bool all = true;
        auto bind = [&](auto &fn, const char *sym) {
            fn = reinterpret_cast<std::remove_reference_t<decltype(fn)>>(dlsym(h, sym));
            if (!fn) {
                all = false;
                R.why = std::string("RCCL symbol missing: ") + sym;
            }
        };
        bind(R.get_unique_id, "ncclGetUniqueId");
        bind(R.init_rank, "ncclCommInitRank");
        bind(R.init_all, "ncclCommInitAll");
        bind(R.destroy, "ncclCommDestroy");
        bind(R.all_reduce, "ncclAllReduce");
        bind(R.reduce, "ncclReduce");
        bind(R.group_start, "ncclGroupStart");
        bind(R.group_end, "ncclGroupEnd");
        bind(R.error_string, "ncclGetErrorString");
        bind(R.async_error, "ncclCommGetAsyncError");
        bind(R.abort, "ncclCommAbort");
        R.ok = all;
    });
    return R;
}

int need_rccl(const char *api) {
    Rccl &R = rccl();
    if (R.ok) return MH_OK;
    return mh_report_error(MH_ERR_UNSUPPORTED, std::string(api) + ": " + R.why);
}

int nccl_fail(const char *api, ncclResult_t r) {
    return mh_report_error(MH_ERR_HIP, std::string(api) + ": " + rccl().error_string(r));
}

}  // namespace

extern "C" {

int mh_comm_unique_id(uint8_t id[MH_COMM_ID_BYTES]) {
    if (!id) return mh_report_error(MH_ERR_INVALID_ARGUMENT, "mh_comm_unique_id: NULL id");
    if (int rc = need_rccl("mh_comm_unique_id")) return rc;
    static_assert(sizeof(ncclUniqueId) == MH_COMM_ID_BYTES, "ncclUniqueId size");
    ncclUniqueId u;
    if (ncclResult_t r = rccl().get_unique_id(&u)) return nccl_fail("mh_comm_unique_id", r);
    memcpy(id, &u, sizeof(u));
    return MH_OK;
}

int mh_comm_create(const uint8_t id[MH_COMM_ID_BYTES], int nranks, int rank, int device, mh_comm **out) {
    if (!id || !out) return mh_report_error(MH_ERR_INVALID_ARGUMENT, "mh_comm_create: NULL argument");
    if (nranks < 1 || rank < 0 || rank >= nranks)
        return mh_report_error(MH_ERR_INVALID_ARGUMENT, "mh_comm_create: rank out of [0, nranks)");
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0)
        return mh_report_error(MH_ERR_NO_DEVICE, "mh_comm_create: no HIP device available");
    if (device < 0 || device >= ndev)
        return mh_report_error(MH_ERR_INVALID_ARGUMENT, "mh_comm_create: device index out of bounds");
    if (int rc = need_rccl("mh_comm_create")) return rc;
    if (hipSetDevice(device) != hipSuccess)
        return mh_report_error(MH_ERR_HIP, "mh_comm_create: hipSetDevice failed");
    ncclUniqueId u;
    memcpy(&u, id, sizeof(u));
    mh_comm *c = new mh_comm;
    c->nranks = nranks;
    c->rank = rank;
    c->device = device;
    if (ncclResult_t r = rccl().init_rank(&c->comm, nranks, u, rank)) {
        delete c;
        return nccl_fail("mh_comm_create", r);
    }
    *out = c;
    return MH_OK;
}

int mh_comm_create_all(int ndev, const int *devices, mh_comm **out) {
    if (ndev < 1 || !devices || !out)
        return mh_report_error(MH_ERR_INVALID_ARGUMENT, "mh_comm_create_all: bad argument");
    int have = 0;
    if (hipGetDeviceCount(&have) != hipSuccess || have == 0)
        return mh_report_error(MH_ERR_NO_DEVICE, "mh_comm_create_all: no HIP device available");
    for (int i = 0; i < ndev; ++i)
        if (devices[i] < 0 || devices[i] >= have)
            return mh_report_error(MH_ERR_INVALID_ARGUMENT, "mh_comm_create_all: device index out of bounds");
    if (int rc = need_rccl("mh_comm_create_all")) return rc;
    std::vector<ncclComm_t> comms(ndev, nullptr);
    if (ncclResult_t r = rccl().init_all(comms.data(), ndev, devices)) return nccl_fail("mh_comm_create_all", r);
    for (int i = 0; i < ndev; ++i) {
        out[i] = new mh_comm;
        out[i]->comm = comms[i];
        out[i]->nranks = ndev;
        out[i]->rank = i;  // ncclCommInitAll: rank i on devices[i]
        out[i]->device = devices[i];
    }
    return MH_OK;
}

int mh_comm_destroy(mh_comm *c) {
    if (!c) return MH_OK;
    if (c->users > 0)  // a scene still holds it (mh_scene_set_comm): destroying it would leave the scene dangling
        return mh_report_error(MH_ERR_INVALID_ARGUMENT, "mh_comm_destroy: the communicator is still attached to " +
                                                            std::to_string(c->users) +
                                                            " scene(s); detach them first (mh_scene_set_comm(scene, NULL))");
    if (c->comm && rccl().ok) {
        (void)hipSetDevice(c->device);
        (void)rccl().destroy(c->comm);
    }
    delete c;
    return MH_OK;
}

int mh_comm_info(const mh_comm *c, int *nranks, int *rank, int *device) {
    if (!c) return mh_report_error(MH_ERR_INVALID_ARGUMENT, "mh_comm_info: NULL communicator");
    if (nranks) *nranks = c->nranks;
    if (rank) *rank = c->rank;
    if (device) *device = c->device;
    return MH_OK;
}

int mh_comm_reduce(mh_comm *const *comms, int n, float *const *bufs, uint64_t count, void *const *streams,
                   int root) {
    if (n < 1 || !comms || !bufs) return mh_report_error(MH_ERR_INVALID_ARGUMENT, "mh_comm_reduce: bad argument");
    for (int i = 0; i < n; ++i)
        if (!comms[i] || !bufs[i]) return mh_report_error(MH_ERR_INVALID_ARGUMENT, "mh_comm_reduce: NULL entry");
    if (root >= comms[0]->nranks)
        return mh_report_error(MH_ERR_INVALID_ARGUMENT, "mh_comm_reduce: root out of [0, nranks)");
    for (int i = 0; i < n; ++i)
        if (comms[i]->aborted)
            return mh_report_error(MH_ERR_HIP, "mh_comm_reduce: the communicator was aborted after an earlier failure "
                                               "of a collective call (create a new one)");
    if (count == 0) return MH_OK;
    if (int rc = need_rccl("mh_comm_reduce")) return rc;
    Rccl &R = rccl();
    // several ranks from one thread: one RCCL group, else the first call
    // could wait for peers this thread has not issued yet
    if (n > 1)
        if (ncclResult_t r = R.group_start()) return nccl_fail("mh_comm_reduce", r);
    ncclResult_t bad = ncclSuccess;
    for (int i = 0; i < n && bad == ncclSuccess; ++i) {
        if (hipSetDevice(comms[i]->device) != hipSuccess) {
            bad = ncclUnhandledCudaError;
            break;
        }
        hipStream_t st = streams ? (hipStream_t)streams[i] : nullptr;
        bad = root < 0 ? R.all_reduce(bufs[i], bufs[i], (size_t)count, ncclFloat32, ncclSum, comms[i]->comm, st)
                       : R.reduce(bufs[i], bufs[i], (size_t)count, ncclFloat32, ncclSum, root, comms[i]->comm, st);
    }
    if (n > 1) {
        ncclResult_t e = R.group_end();
        if (bad == ncclSuccess) bad = e;
    }
    if (bad != ncclSuccess) return nccl_fail("mh_comm_reduce", bad);
    return MH_OK;
}

}  // extern "C"

// ---- failure handling of the in-call collectives (mh_api.hip) ----
// A rank that fails inside a MH_FLAG_REDUCE call returns before it has issued
// every collective of the call, while its peers have queued theirs: the
// peers' streams can then never drain.  So (1) a rank waits for its stream
// through comm_wait, which polls the stream and the communicator's async error
// with a deadline (MH_COMM_TIMEOUT_S, default 1800 s) instead of blocking in
// hipStreamSynchronize, and (2) a rank whose call fails aborts its
// communicator (comm_abort), as does a rank whose wait runs out: every rank
// then returns an error, and every later collective on that communicator
// fails at once instead of pairing with the wrong collective of a peer.
void comm_abort(mh_comm *c) {
    if (!c || c->aborted) return;
    c->aborted = true;
    if (c->comm && rccl().ok) {
        (void)hipSetDevice(c->device);
        (void)rccl().abort(c->comm);
    }
    c->comm = nullptr;
}

int comm_wait(mh_comm *c, hipStream_t st, const char *api) {
    static const double timeout_s = [] {
        const char *e = getenv("MH_COMM_TIMEOUT_S");
        return e ? std::max(0.001, atof(e)) : 1800.0;
    }();
    const auto t0 = std::chrono::steady_clock::now();
    for (uint32_t it = 0;; ++it) {
        const hipError_t q = hipStreamQuery(st);
        if (q == hipSuccess) return MH_OK;
        if (q != hipErrorNotReady) {
            comm_abort(c);
            return mh_report_error(MH_ERR_HIP, std::string(api) + ": " + hipGetErrorString(q));
        }
        if (c && !c->aborted && c->comm && rccl().ok) {
            ncclResult_t r = ncclSuccess;
            if (rccl().async_error(c->comm, &r) == ncclSuccess && r != ncclSuccess && r != ncclInProgress) {
                comm_abort(c);
                return mh_report_error(MH_ERR_HIP, std::string(api) + ": a collective failed: " + rccl().error_string(r));
            }
        }
        const double dt = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
        if (dt > timeout_s) {
            comm_abort(c);
            return mh_report_error(MH_ERR_HIP, std::string(api) + ": the call's collectives did not complete within " +
                                                   std::to_string(timeout_s) + " s (a peer rank failed?); "
                                                   "the communicator was aborted");
        }
        if (it < 2000) std::this_thread::yield();
        else std::this_thread::sleep_for(std::chrono::microseconds(50));
    }
}

void comm_attach(mh_comm *c, int delta) {
    if (c) c->users += delta;
}

// in-call reduction of one rank (mh_api.hip: MH_FLAG_REDUCE / MH_FLAG_REDUCE_ROOT)
int comm_reduce_one(mh_comm *c, int device, float *buf, uint64_t count, hipStream_t st, int root) {
    if (c->device != device)
        return mh_report_error(MH_ERR_INVALID_ARGUMENT, "MH_FLAG_REDUCE: the communicator's device is not the scene's");
    void *sp = st;
    int rc = mh_comm_reduce(&c, 1, &buf, count, &sp, root);
    // test hook (tests/test_gpu_comm.py): a one-rank sum leaves the data as it
    // is, so a wrong extent, buffer or root would go unseen; MH_TEST_COMM_SCALE
    // doubles exactly the reduced extent (buf += buf) at world size 1
    if (rc == MH_OK && c->nranks == 1 && count && getenv("MH_TEST_COMM_SCALE"))
        if (mh::launch_accumulate(buf, buf, count, st) != hipSuccess)
            rc = mh_report_error(MH_ERR_HIP, "MH_TEST_COMM_SCALE: launch failed");
    return rc;
}
