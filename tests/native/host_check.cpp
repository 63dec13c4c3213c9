// host_check.cpp — drives the host-only C++ of libppgpu under AddressSanitizer + UBSan and
// ThreadSanitizer (SURVEY §5 "ASan/TSan on the C++ CPU path").  No GPU is
// touched: every call below is host code (CreateIndex over zlib, IndexIO, validate, partition,
// from_points, the shared-memory communicator and its two-phase gather with failing ranks).
// The reference ships real races in the same roles (LazyFileReader.cs:41-97 shares a FileStream
// across tasks; BatchedFASTQ.cs:76-77 mutates a task list from continuations), which is what the
// threaded parts here are checked for.
//
//   host_check <golden dir> <scratch dir>     exit status 0 = every check passed
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <string>
#include <thread>
#include <vector>

#include "../../include/ppgpu.h"
#include "../../parallelparsing_amd/csrc/ppg_host.h"

static std::atomic<int> failures{0};
#define CHECK(c)                                                                  \
    do {                                                                          \
        if (!(c)) {                                                               \
            fprintf(stderr, "CHECK failed: %s (%s:%d)\n", #c, __FILE__, __LINE__); \
            failures++;                                                           \
        }                                                                         \
    } while (0)

static std::vector<uint8_t> slurp(const std::string &path) {
    std::vector<uint8_t> b;
    FILE *f = fopen(path.c_str(), "rb");
    if (!f) return b;
    uint8_t buf[1 << 16];
    size_t n;
    while ((n = fread(buf, 1, sizeof buf, f)) > 0) b.insert(b.end(), buf, buf + n);
    fclose(f);
    return b;
}

// CreateIndex (mem and file), Serialize -> Deserialize round trip, from_points, validate, partition
static void check_index(const std::string &gz_path, uint32_t chunk, const std::string &scratch, int tag = 0) {
    std::vector<uint8_t> gz = slurp(gz_path);
    CHECK(!gz.empty());
    ppg_index *a = nullptr, *b = nullptr, *c = nullptr, *d = nullptr;
    CHECK(ppg_index_build_mem(gz.data(), (int64_t)gz.size(), chunk, &a) == PPG_OK);
    CHECK(ppg_index_build_file(gz_path.c_str(), chunk, &b) == PPG_OK);
    if (!a || !b) return;
    const int32_t n = ppg_index_count(a);
    CHECK(n == ppg_index_count(b) && n >= 2);
    const std::string gzi = scratch + "/hc" + std::to_string(tag) + ".gzi";
    CHECK(ppg_index_serialize(a, gzi.c_str()) == PPG_OK);
    CHECK(ppg_index_deserialize(gzi.c_str(), &c) == PPG_OK);
    std::vector<int64_t> out(n), in(n);
    std::vector<int32_t> bits(n), ol(n);
    std::vector<uint8_t> win((size_t)n * PPG_WINSIZE), offs;
    for (int32_t i = 0; i < n; i++) {
        int64_t o2, i2;
        int32_t b2, l2;
        CHECK(ppg_index_point(a, i, &out[i], &in[i], &bits[i], &ol[i]) == PPG_OK);
        CHECK(ppg_index_point(c, i, &o2, &i2, &b2, &l2) == PPG_OK);
        CHECK(o2 == out[i] && i2 == in[i] && b2 == bits[i] && l2 == ol[i]);
        CHECK(memcmp(ppg_index_window(a, i), ppg_index_window(c, i), PPG_WINSIZE) == 0);
        memcpy(win.data() + (size_t)i * PPG_WINSIZE, ppg_index_window(a, i), PPG_WINSIZE);
        const uint8_t *p = ppg_index_offset(a, i);
        offs.insert(offs.end(), p, p + ol[i]);
        CHECK(ol[i] == 0 || memcmp(p, ppg_index_offset(c, i), (size_t)ol[i]) == 0);
    }
    offs.push_back(0);
    CHECK(ppg_index_from_points(n, out.data(), in.data(), bits.data(), win.data(), ol.data(), offs.data(),
                                ppg_index_chunk_max_bytes(a), &d) == PPG_OK);
    CHECK(d && ppg_index_count(d) == n);
    CHECK(ppg_index_validate(a, 0, n - 1) == PPG_OK);
    CHECK(ppg_index_validate(a, 0, n) == PPG_ARG_ERROR);
    for (int32_t R : {1, 2, 3, 8}) {
        std::vector<int32_t> bounds((size_t)R + 1);
        CHECK(ppg_partition(a, 0, n - 1, R, bounds.data()) == PPG_OK);
        CHECK(bounds[0] == 0 && bounds[(size_t)R] == n - 1);
        for (int32_t r = 0; r < R; r++) CHECK(bounds[(size_t)r] <= bounds[(size_t)r + 1]);
    }
    // a truncated file is an error, not a crash
    ppg_index *e = nullptr;
    CHECK(ppg_index_build_mem(gz.data(), (int64_t)gz.size() / 2, chunk, &e) != PPG_OK && e == nullptr);
    ppg_index_free(a);
    ppg_index_free(b);
    ppg_index_free(c);
    ppg_index_free(d);
    unlink(gzi.c_str());
}

// the shared-memory communicator with `world` ranks as threads: rendezvous, then several rounds of
// the two-phase count gather in which ranks fail in turn (no context: ARG_ERROR) -- every rank
// must return the same status every round, none may hang
static void check_comm(const std::string &gz_path, uint32_t chunk, int world, int rounds) {
    ppg_index *ix = nullptr;
    CHECK(ppg_index_build_file(gz_path.c_str(), chunk, &ix) == PPG_OK);
    if (!ix) return;
    char name[64];
    snprintf(name, sizeof name, "/ppg_hc_%d_%d", (int)getpid(), world);
    std::vector<std::vector<int>> got((size_t)world);
    std::vector<std::thread> th;
    std::atomic<int> opened{0};
    for (int r = 0; r < world; r++) {
        th.emplace_back([&, r] {
            ppg_comm *c = nullptr;
            if (ppg_comm_init_host(world, r, name, &c) != PPG_OK) return;
            opened++;
            int32_t rank = -1, nranks = -1;
            CHECK(ppg_comm_rank(c, &rank, &nranks) == PPG_OK && rank == r && nranks == world);
            const int32_t m = ppg_index_count(ix) - 1;
            std::vector<int64_t> counts((size_t)m), bases((size_t)m);
            for (int k = 0; k < rounds; k++) {
                int64_t tot = -1;
                // round k: rank k % world passes no index as well
                const ppg_index *mine = (r == k % world) ? nullptr : ix;
                got[(size_t)r].push_back(ppg_dist_decompress_all(nullptr, c, mine, gz_path.c_str(), 0, counts.data(),
                                                                 bases.data(), &tot));
                // a rank with no shard (NULL) joins the gather too
                got[(size_t)r].push_back(ppg_shard_gather_counts(nullptr, c, nullptr, nullptr, nullptr, &tot));
            }
            ppg_comm_free(c);
        });
    }
    for (auto &t : th) t.join();
    CHECK(opened == world);
    for (int r = 0; r < world; r++) {
        CHECK(got[(size_t)r].size() == (size_t)(2 * rounds));
        for (size_t i = 0; i < got[(size_t)r].size(); i++) CHECK(got[(size_t)r][i] == PPG_ARG_ERROR);
    }
    ppg_index_free(ix);
}

// ppg_comm_alltoallv over the host transport with `world` ranks as threads, host buffers: uneven
// and zero counts and one pair large enough for several rounds of the shared slots; then
// ppg_pairs_check with no shards on every rank (every rank joins the status gather and fails alike)
static void check_alltoallv(int world) {
    char name[64];
    snprintf(name, sizeof name, "/ppg_hc_a2a_%d_%d", (int)getpid(), world);
    std::vector<int64_t> m((size_t)world * world);
    for (int a = 0; a < world; a++)
        for (int b = 0; b < world; b++) m[(size_t)a * world + b] = (a * 7 + b * 13) % 11 * 97;
    m[(size_t)world - 1] = 1500000;   // rank 0 -> last rank: several rounds
    m[(size_t)(world - 1) * world] = 0;
    std::vector<std::thread> th;
    std::atomic<int> ok{0};
    for (int r = 0; r < world; r++) {
        th.emplace_back([&, r] {
            ppg_comm *c = nullptr;
            if (ppg_comm_init_host(world, r, name, &c) != PPG_OK) return;
            std::vector<int64_t> send, want;
            for (int d = 0; d < world; d++)
                for (int64_t i = 0; i < m[(size_t)r * world + d]; i++) send.push_back(r * 10000000LL + d * 1000000LL + i);
            for (int s2 = 0; s2 < world; s2++)
                for (int64_t i = 0; i < m[(size_t)s2 * world + r]; i++) want.push_back(s2 * 10000000LL + r * 1000000LL + i);
            std::vector<int64_t> recv(want.size() + 1, -7);
            int64_t dummy = 0;
            const int rc = ppg_comm_alltoallv(c, send.empty() ? &dummy : send.data(), recv.data(), m.data(), 0);
            CHECK(rc == PPG_OK);
            CHECK(std::equal(want.begin(), want.end(), recv.begin()));
            ppg_pairs *p = nullptr;
            CHECK(ppg_pairs_create(&p) == PPG_OK);
            ppg_pair_result res;
            CHECK(ppg_pairs_check(p, nullptr, nullptr, c, &res) == PPG_ARG_ERROR);
            ppg_pairs_free(p);
            ppg_comm_free(c);
            ok++;
        });
    }
    for (auto &t : th) t.join();
    CHECK(ok == world);
}

// The RCCL grouped send/recv of ppg_comm_alltoallv with fake entry points (a failed
// ncclSend / ncclRecv returned with the group still open).  Whichever call fails -- the k-th send or
// recv, or ncclGroupEnd itself -- the group is closed exactly once, nothing is enqueued after the
// failure, and the status is PPG_DEVICE_ERROR; a failed ncclGroupStart opens nothing.
namespace fake_rccl {
static int calls, fail_at, starts, ends, after_fail;
static bool failed, fail_start, fail_end;
static ncclResult_t step() {
    if (failed) after_fail++;
    if (++calls == fail_at) { failed = true; return ncclUnhandledCudaError; }
    return ncclSuccess;
}
static ncclResult_t send(const void *, size_t, ncclDataType_t, int, ncclComm_t, hipStream_t) { return step(); }
static ncclResult_t recv(void *, size_t, ncclDataType_t, int, ncclComm_t, hipStream_t) { return step(); }
static ncclResult_t gstart() { starts++; return fail_start ? ncclInternalError : ncclSuccess; }
static ncclResult_t gend() { ends++; return fail_end ? ncclInternalError : ncclSuccess; }
static const char *err(ncclResult_t) { return "fake"; }
}  // namespace fake_rccl

static void check_grouped_p2p() {
    namespace F = fake_rccl;
    const int32_t R = 4, me = 1;
    std::vector<int64_t> m((size_t)R * R, 5), sd((size_t)R + 1), rd((size_t)R + 1);
    for (int32_t q = 0; q < R; q++) {
        sd[(size_t)q + 1] = sd[(size_t)q] + m[(size_t)me * R + q];
        rd[(size_t)q + 1] = rd[(size_t)q] + m[(size_t)q * R + me];
    }
    std::vector<int64_t> snd((size_t)sd[R]), rcv((size_t)rd[R]);
    const CommP2P f{F::send, F::recv, F::gstart, F::gend, F::err};
    const int total = 2 * (R - 1);   // one send and one recv per peer
    for (int mode = 0; mode <= total + 2; mode++) {
        F::calls = F::starts = F::ends = F::after_fail = 0;
        F::failed = false;
        F::fail_at = mode >= 1 && mode <= total ? mode : 0;
        F::fail_start = mode == total + 1;
        F::fail_end = mode == total + 2;
        const int rc = comm_grouped_p2p(f, nullptr, nullptr, snd.data(), rcv.data(), m.data(), R, me, sd.data(), rd.data());
        CHECK(rc == (mode == 0 ? PPG_OK : PPG_DEVICE_ERROR));
        CHECK(F::starts == 1);
        CHECK(F::ends == (F::fail_start ? 0 : 1));      // always closed once, unless never opened
        CHECK(F::after_fail == 0);                      // nothing enqueued after the failure
        CHECK(F::calls == (F::fail_start ? 0 : F::fail_at ? F::fail_at : total));
    }
}

int main(int argc, char **argv) {
    if (argc < 3) {
        fprintf(stderr, "usage: host_check <golden dir> <scratch dir>\n");
        return 2;
    }
    const std::string g = argv[1], scratch = argv[2];
    const struct { const char *name; uint32_t chunk; } cases[] = {
        {"l6_c20", 20}, {"l6_c200", 200}, {"l1_c150", 150}, {"l9_c300", 300}, {"fixed_c100", 100},
        {"huffonly_c20", 20}, {"rle_c100", 100}, {"stored_c50", 50}, {"memlevel1_c10", 10}, {"pigz_c100", 100},
        {"crlf_c100", 100}, {"malformed_c40", 40}, {"nul_c60", 60}, {"plusline_c50", 50}, {"short_reads_c30", 30},
        {"long_reads_c10", 10}, {"one_record", 10000}};
    for (const auto &c : cases) check_index(g + "/" + c.name + ".gz", c.chunk, scratch);
    // CreateIndex in parallel threads over the same file (the reference decodes chunks from many
    // threads; each ppg call owns its zlib stream, Core.cs:136)
    {
        std::vector<std::thread> th;
        for (int t = 0; t < 4; t++) th.emplace_back([&, t] { check_index(g + "/l6_c200.gz", 200, scratch, 1 + t); });
        for (auto &t : th) t.join();
    }
    for (int world : {2, 3, 5}) check_comm(g + "/l6_c200.gz", 200, world, 4);
    for (int world : {2, 3}) check_alltoallv(world);
    check_grouped_p2p();
    printf("host_check: %s (%d failures)\n", failures ? "FAILED" : "ok", failures.load());
    return failures ? 1 : 0;
}
