// gac_comm.hip -- the -nranks collective of the C ABI (SURVEY.md §8(b):
// gac_allgather, "wraps ncclAllGather").  One process per GPU of one node;
// two backends behind one call:
//
//   GAC_COMM_RCCL  ncclAllGather over xGMI.  librccl is opened at run time
//                  (dlopen: a tool that never gathers does not pay for
//                  loading it); rank 0's ncclUniqueId reaches the others
//                  through the host backend; the payload goes host -> HBM,
//                  one ncclAllGather, HBM -> host, on a stream of the
//                  communicator's device.
//   GAC_COMM_HOST  files next to the caller's rendezvous prefix (the node's
//                  page cache): each rank writes its part, a barrier, every
//                  rank reads all parts, a barrier, each deletes its own.
//                  No device: the CPU tests, and ranks that share a GPU
//                  (RCCL refuses two ranks on one device).
//
// Barriers are O_APPEND counter files: a rank appends one byte to
// <prefix>.b<k> and waits for the file to reach nranks bytes; it then appends
// to <prefix>.l<k>, and the rank whose byte lands last there removes both
// (every rank has left the wait by then).  A wait gives up after `timeout`
// seconds, or when the caller's liveness callback says a peer has failed.
#include <dlfcn.h>
#include <errno.h>
#include <fcntl.h>
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/stat.h>
#include <time.h>
#include <unistd.h>

#include <string>
#include <vector>

#include "gachain.h"
#include "host/gac_host.h"

namespace {

// ncclAllGather and friends, resolved from librccl at run time
struct Rccl {
    void *so = nullptr;
    ncclResult_t (*get_unique_id)(ncclUniqueId *) = nullptr;
    ncclResult_t (*comm_init_rank)(ncclComm_t *, int, ncclUniqueId, int) = nullptr;
    ncclResult_t (*all_gather)(const void *, void *, size_t, ncclDataType_t, ncclComm_t, hipStream_t) = nullptr;
    ncclResult_t (*comm_destroy)(ncclComm_t) = nullptr;
    const char *(*error_string)(ncclResult_t) = nullptr;
};

int rccl_load(Rccl &r) {
    if (r.so) return GAC_OK;
    const char *names[] = {"librccl.so.1", "librccl.so", "/opt/rocm/lib/librccl.so.1"};
    for (const char *n : names)
        if ((r.so = dlopen(n, RTLD_NOW | RTLD_LOCAL)) != nullptr) break;
    if (!r.so) return gac_fail(GAC_E_STATE, "gac_comm: librccl not found (%s)", dlerror());
    r.get_unique_id = (decltype(r.get_unique_id))dlsym(r.so, "ncclGetUniqueId");
    r.comm_init_rank = (decltype(r.comm_init_rank))dlsym(r.so, "ncclCommInitRank");
    r.all_gather = (decltype(r.all_gather))dlsym(r.so, "ncclAllGather");
    r.comm_destroy = (decltype(r.comm_destroy))dlsym(r.so, "ncclCommDestroy");
    r.error_string = (decltype(r.error_string))dlsym(r.so, "ncclGetErrorString");
    if (!r.get_unique_id || !r.comm_init_rank || !r.all_gather || !r.comm_destroy || !r.error_string)
        return gac_fail(GAC_E_STATE, "gac_comm: librccl lacks the ncclAllGather API");
    return GAC_OK;
}

double mono_s() {
    struct timespec t;
    clock_gettime(CLOCK_MONOTONIC, &t);
    return t.tv_sec + 1e-9 * t.tv_nsec;
}

}  // namespace

struct gac_comm {
    std::string prefix;
    int n = 1, me = 0, device = -1, backend = GAC_COMM_HOST;
    double timeout = 600.0;
    int (*alive)(int rank, void *user) = nullptr;
    void *user = nullptr;
    int64_t seq = 0;  // calls made (file names)
    int64_t bar = 0;  // barriers passed
    Rccl rc;
    ncclComm_t nc = nullptr;
    hipStream_t st = nullptr;
    double init_s = 0;  // RCCL communicator set-up time (gac_comm_stats)
};

namespace {

std::string part_name(const gac_comm *c, int64_t s, int r) {
    return c->prefix + ".c" + std::to_string(s) + ".r" + std::to_string(r);
}

// wait until `path` holds at least `want` bytes (a peer's part: its rename
// makes it appear whole), polling with a growing pause
int wait_size(const gac_comm *c, const std::string &path, int64_t want) {
    const double t0 = mono_s();
    struct timespec ts = {0, 20000};
    for (int it = 0;; ++it) {
        struct stat sb;
        if (stat(path.c_str(), &sb) == 0 && sb.st_size >= want) return GAC_OK;
        if ((it & 63) == 63) {
            if (mono_s() - t0 > c->timeout)
                return gac_fail(GAC_E_STATE, "gac_comm: rank %d: no %s after %.0f s", c->me,
                                path.c_str(), c->timeout);
            for (int peer = 0; c->alive && peer < c->n; ++peer)
                if (peer != c->me && !c->alive(peer, c->user))
                    return gac_fail(GAC_E_STATE, "gac_comm: rank %d: peer rank %d failed", c->me, peer);
            if (ts.tv_nsec < 1000000) ts.tv_nsec *= 2;
        }
        nanosleep(&ts, nullptr);
    }
}

int append_byte(const std::string &path, int64_t *pos) {
    const int fd = open(path.c_str(), O_WRONLY | O_CREAT | O_APPEND, 0644);
    if (fd < 0) return gac_fail(GAC_E_IO, "gac_comm: can't open %s: %s", path.c_str(), strerror(errno));
    const char b = 1;
    const ssize_t w = write(fd, &b, 1);
    const off_t at = lseek(fd, 0, SEEK_CUR);  // (O_APPEND: just past this rank's byte)
    close(fd);
    if (w != 1) return gac_fail(GAC_E_IO, "gac_comm: can't append to %s", path.c_str());
    if (pos) *pos = (int64_t)at;
    return GAC_OK;
}

int barrier(gac_comm *c) {
    if (c->n == 1) return GAC_OK;
    const int64_t k = c->bar++;
    const std::string b = c->prefix + ".b" + std::to_string(k), l = c->prefix + ".l" + std::to_string(k);
    int rc = append_byte(b, nullptr);
    if (rc != GAC_OK) return rc;
    if ((rc = wait_size(c, b, c->n)) != GAC_OK) return rc;
    int64_t pos = 0;
    if ((rc = append_byte(l, &pos)) != GAC_OK) return rc;
    if (pos == c->n) {  // the last to leave: nobody waits on either file now
        unlink(b.c_str());
        unlink(l.c_str());
    }
    return GAC_OK;
}

int write_part(const gac_comm *c, int64_t s, const void *p, size_t bytes) {
    const std::string f = part_name(c, s, c->me), tmp = f + ".tmp";
    FILE *o = fopen(tmp.c_str(), "wb");
    if (!o) return gac_fail(GAC_E_IO, "gac_comm: can't write %s: %s", tmp.c_str(), strerror(errno));
    const bool ok = (bytes == 0 || fwrite(p, 1, bytes, o) == bytes);
    if (fclose(o) != 0 || !ok || rename(tmp.c_str(), f.c_str()) != 0)
        return gac_fail(GAC_E_IO, "gac_comm: can't write %s", f.c_str());
    return GAC_OK;
}

// the host backend's gather of variable parts: out = parts in rank order
int host_gatherv(gac_comm *c, const void *send, size_t bytes, std::vector<char> &out,
                 std::vector<size_t> &counts) {
    const int64_t s = c->seq++;
    counts.assign(c->n, 0);
    int rc;
    if ((rc = write_part(c, s, send, bytes)) != GAC_OK) return rc;
    if ((rc = barrier(c)) != GAC_OK) return rc;
    size_t total = 0;
    for (int r = 0; r < c->n; ++r) {
        struct stat sb;
        const std::string f = part_name(c, s, r);
        if (stat(f.c_str(), &sb) != 0) return gac_fail(GAC_E_IO, "gac_comm: %s missing", f.c_str());
        counts[r] = (size_t)sb.st_size;
        total += counts[r];
    }
    out.resize(total);
    size_t at = 0;
    for (int r = 0; r < c->n; ++r) {
        if (r == c->me) {
            if (bytes) memcpy(out.data() + at, send, bytes);
        } else if (counts[r]) {
            const std::string f = part_name(c, s, r);
            FILE *in = fopen(f.c_str(), "rb");
            const bool ok = in && fread(out.data() + at, 1, counts[r], in) == counts[r];
            if (in) fclose(in);
            if (!ok) return gac_fail(GAC_E_IO, "gac_comm: can't read %s", f.c_str());
        }
        at += counts[r];
    }
    if ((rc = barrier(c)) != GAC_OK) return rc;  // (every rank has read every part)
    unlink(part_name(c, s, c->me).c_str());
    return GAC_OK;
}

#define NCCHK(x)                                                                                  \
    do {                                                                                          \
        const ncclResult_t r_ = (x);                                                              \
        if (r_ != ncclSuccess)                                                                    \
            return gac_fail(GAC_E_HIP, "gac_comm: %s: %s", #x, c->rc.error_string(r_));           \
    } while (0)
#define HCHK(x)                                                                                   \
    do {                                                                                          \
        const hipError_t e_ = (x);                                                                \
        if (e_ != hipSuccess) return gac_fail(GAC_E_HIP, "gac_comm: %s: %s", #x, hipGetErrorString(e_)); \
    } while (0)

int rccl_open(gac_comm *c) {
    const double t0 = mono_s();
    int rc = rccl_load(c->rc);
    if (rc != GAC_OK) return rc;
    HCHK(hipSetDevice(c->device));
    ncclUniqueId id;
    memset(&id, 0, sizeof(id));
    if (c->me == 0) NCCHK(c->rc.get_unique_id(&id));
    std::vector<char> all;
    std::vector<size_t> cnt;
    if ((rc = host_gatherv(c, &id, c->me == 0 ? sizeof(id) : 0, all, cnt)) != GAC_OK) return rc;
    if (cnt[0] != sizeof(id)) return gac_fail(GAC_E_STATE, "gac_comm: no RCCL id from rank 0");
    memcpy(&id, all.data(), sizeof(id));
    HCHK(hipStreamCreateWithFlags(&c->st, hipStreamNonBlocking));
    NCCHK(c->rc.comm_init_rank(&c->nc, c->n, id, c->me));
    c->init_s = mono_s() - t0;
    return GAC_OK;
}

// ncclAllGather of `bytes` per rank from host `send` into host `recv`
int rccl_gather(gac_comm *c, const void *send, size_t bytes, void *recv) {
    if (bytes == 0) return GAC_OK;
    HCHK(hipSetDevice(c->device));
    void *d = nullptr;
    HCHK(hipMalloc(&d, bytes * (c->n + 1)));
    char *dsend = (char *)d + bytes * c->n, *drecv = (char *)d;
    hipError_t e = hipMemcpyAsync(dsend, send, bytes, hipMemcpyHostToDevice, c->st);
    ncclResult_t r = ncclSuccess;
    if (e == hipSuccess) r = c->rc.all_gather(dsend, drecv, bytes, ncclChar, c->nc, c->st);
    if (e == hipSuccess && r == ncclSuccess)
        e = hipMemcpyAsync(recv, drecv, bytes * c->n, hipMemcpyDeviceToHost, c->st);
    if (e == hipSuccess && r == ncclSuccess) e = hipStreamSynchronize(c->st);
    hipFree(d);
    if (r != ncclSuccess) return gac_fail(GAC_E_HIP, "gac_comm: ncclAllGather: %s", c->rc.error_string(r));
    if (e != hipSuccess) return gac_fail(GAC_E_HIP, "gac_comm: %s", hipGetErrorString(e));
    return GAC_OK;
}

}  // namespace

extern "C" int gac_comm_open(const char *rendezvous, int nranks, int rank, int device, int backend,
                             double timeout_s, int (*alive)(int rank, void *user), void *user,
                             gac_comm **out) {
    gac_clear_error();
    if (!out || !rendezvous || !*rendezvous || nranks < 1 || rank < 0 || rank >= nranks ||
        (backend != GAC_COMM_AUTO && backend != GAC_COMM_HOST && backend != GAC_COMM_RCCL))
        return gac_fail(GAC_E_ARG, "gac_comm_open: bad argument");
    *out = nullptr;
    if (backend == GAC_COMM_AUTO) {
        // GAC_COMM=rccl|host chooses; else RCCL when this rank names a device
        const char *e = getenv("GAC_COMM");
        backend = e && !strcmp(e, "host") ? GAC_COMM_HOST
                  : e && !strcmp(e, "rccl") ? GAC_COMM_RCCL
                  : device >= 0 ? GAC_COMM_RCCL : GAC_COMM_HOST;
    }
    if (backend == GAC_COMM_RCCL && device < 0)
        return gac_fail(GAC_E_ARG, "gac_comm_open: the RCCL backend needs a device");
    gac_comm *c = new gac_comm();
    c->prefix = rendezvous;
    c->n = nranks;
    c->me = rank;
    c->device = device;
    c->backend = backend;
    c->timeout = timeout_s > 0 ? timeout_s : 600.0;
    c->alive = alive;
    c->user = user;
    if (backend == GAC_COMM_RCCL) {
        const int rc = rccl_open(c);
        if (rc != GAC_OK) {
            gac_comm_close(c);
            return rc;
        }
    }
    *out = c;
    return GAC_OK;
}

extern "C" int gac_comm_backend(const gac_comm *c) { return c ? c->backend : -1; }

extern "C" double gac_comm_init_seconds(const gac_comm *c) { return c ? c->init_s : 0.0; }

extern "C" int gac_allgather(gac_comm *c, const void *send, size_t bytes, void *recv) {
    gac_clear_error();
    if (!c || (bytes && (!send || !recv))) return gac_fail(GAC_E_ARG, "gac_allgather: bad argument");
    if (c->n == 1) {
        if (bytes) memmove(recv, send, bytes);
        return GAC_OK;
    }
    if (c->backend == GAC_COMM_RCCL) return rccl_gather(c, send, bytes, recv);
    std::vector<char> all;
    std::vector<size_t> cnt;
    const int rc = host_gatherv(c, send, bytes, all, cnt);
    if (rc != GAC_OK) return rc;
    for (int r = 0; r < c->n; ++r)
        if (cnt[r] != bytes)
            return gac_fail(GAC_E_ARG, "gac_allgather: rank %d sent %zu bytes, rank %d %zu", r, cnt[r],
                            c->me, bytes);
    if (bytes) memcpy(recv, all.data(), all.size());
    return GAC_OK;
}

extern "C" int gac_allgatherv(gac_comm *c, const void *send, size_t bytes, void **recv, size_t *counts) {
    gac_clear_error();
    if (!c || !recv || !counts || (bytes && !send)) return gac_fail(GAC_E_ARG, "gac_allgatherv: bad argument");
    *recv = nullptr;
    std::vector<char> all;
    std::vector<size_t> cnt(c->n, 0);
    if (c->n == 1) {
        all.assign((const char *)send, (const char *)send + bytes);
        cnt[0] = bytes;
    } else if (c->backend == GAC_COMM_RCCL) {
        // counts first, then every part padded to the largest
        std::vector<uint64_t> sz(c->n);
        uint64_t mine = bytes;
        int rc = rccl_gather(c, &mine, sizeof(mine), sz.data());
        if (rc != GAC_OK) return rc;
        uint64_t mx = 0;
        for (int r = 0; r < c->n; ++r) mx = sz[r] > mx ? sz[r] : mx;
        std::vector<char> pad(mx), got(mx * c->n);
        if (bytes) memcpy(pad.data(), send, bytes);
        if ((rc = rccl_gather(c, pad.data(), mx, got.data())) != GAC_OK) return rc;
        for (int r = 0; r < c->n; ++r) {
            cnt[r] = sz[r];
            all.insert(all.end(), got.begin() + r * mx, got.begin() + r * mx + sz[r]);
        }
    } else {
        const int rc = host_gatherv(c, send, bytes, all, cnt);
        if (rc != GAC_OK) return rc;
    }
    void *p = malloc(all.size() ? all.size() : 1);
    if (!p) return gac_fail(GAC_E_IO, "gac_allgatherv: out of host memory");
    if (!all.empty()) memcpy(p, all.data(), all.size());
    for (int r = 0; r < c->n; ++r) counts[r] = cnt[r];
    *recv = p;
    return GAC_OK;
}

extern "C" int gac_comm_barrier(gac_comm *c) {
    gac_clear_error();
    if (!c) return gac_fail(GAC_E_ARG, "gac_comm_barrier: bad argument");
    return barrier(c);
}

extern "C" void gac_comm_close(gac_comm *c) {
    if (!c) return;
    if (c->nc) c->rc.comm_destroy(c->nc);
    if (c->st) hipStreamDestroy(c->st);
    // (librccl stays loaded: unloading a library with live helper threads
    // is not safe)
    delete c;
}
