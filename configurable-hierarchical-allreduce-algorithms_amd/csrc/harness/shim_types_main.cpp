// shim_types_main.cpp -- the reference-signature binding (csrc/shim/chiara_mpi_shim.cpp) over MPI's
// predefined datatype x op table.
//
//   mpiexec -n 4 bin/chiara_shim_types
//
// The reference is generic over MPI_Datatype and MPI_Op (all_reduce_radix_batch.cpp:202-204, sizes
// from MPI_Type_size at :234-277; reduce_scatter_radix_batch.cpp:200-202; allreduce_ring.cpp:3).
// For every (type, op) pair this calls the shim's all_reduce_radix_batch, reduce_scatter_radix_batch
// and MPICH_Allreduce_ring with the reference's own C++ signatures and compares with the MPI
// library's MPI_Allreduce / MPI_Reduce_scatter_block on the same inputs.  The expectation comes from
// MPICH itself: a pair MPICH's MPI_Reduce_local accepts must succeed through the shim with the
// library's result (exact: integer data, and floats holding small integers, so every association
// rounds the same); a pair it rejects must come back as an MPI error class, as must user ops and
// the long-double types.  The MAXLOC / MINLOC pair types and the C complex types are in the table:
// buffers are laid out at MPI's extent (MPI_DOUBLE_INT: 16 B an element, of which 12 are data).
// Prints one JSON line; exit status 0 = all agree.
#include <dlfcn.h>
#include <mpi.h>

#include <cstdlib>

#include <cstdint>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

int all_reduce_radix_batch(char* sendbuf, char* recvbuf, int count, MPI_Datatype datatype, MPI_Op op, MPI_Comm comm,
                           int k, int b);
int reduce_scatter_radix_batch(const void* sendbuf, void* recvbuf, MPI_Aint recvcount, MPI_Datatype datatype,
                               MPI_Op op, MPI_Comm comm, int k, int b);
int MPICH_Allreduce_ring(const char* sendbuf, char* recvbuf, int count, MPI_Datatype datatype, MPI_Op op,
                         MPI_Comm comm);
int allgather_radix_batch(char* sendbuf, int sendcount, MPI_Datatype datatype, char* recvbuf, MPI_Comm comm, int k,
                          int b);
int MPICH_Allreduce_k_reduce_scatter_allgather(const char* sendbuf, char* recvbuf, int count, MPI_Datatype datatype,
                                               MPI_Op op, MPI_Comm comm, int k, int single_phase_recv);
// the shim's user-op binding (csrc/shim/chiara_mpi_shim.cpp); the launcher type is chiara.h's chr_user_reduce_fn
typedef int (*user_reduce_fn)(void*, const void*, const void* const*, int, size_t, int, int, void*, void*);
extern "C" int chiara_shim_op_bind(MPI_Op op, user_reduce_fn fn, void* ctx);
extern "C" int chiara_shim_op_unbind(MPI_Op op);

namespace {

uint64_t mix(uint64_t x) {
    x += 0x9E3779B97F4A7C15ull;
    x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
    x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
    return x ^ (x >> 31);
}

struct TypeCase {
    MPI_Datatype t;
    const char* name;
    int kind;  // 0 integer (random bits), 1 float, 2 double, 3 bool (0/1), 4 pair {value; int}, 5 complex
    int vsize; // pairs: bytes of the value (4 float / 8 double / 8 long / 4 int / 2 short); complex: of a part
    bool vfloat;
};

void put_small(char* p, int v, int vsize, bool vfloat) {
    if (vfloat && vsize == 4) {
        const float f = (float)v;
        std::memcpy(p, &f, 4);
    } else if (vfloat) {
        const double d = (double)v;
        std::memcpy(p, &d, 8);
    } else {
        const int64_t w = v;
        std::memcpy(p, &w, vsize);  // little endian: the low bytes
    }
}

void fill(std::vector<char>& buf, int n, const TypeCase& tc, int tsize, int rank, int salt) {
    buf.assign((size_t)n * tsize, 0);
    for (int i = 0; i < n; ++i) {
        const uint64_t u = mix(((uint64_t)rank << 40) ^ ((uint64_t)salt << 20) ^ (uint64_t)i);
        char* p = buf.data() + (size_t)i * tsize;
        if (tc.kind == 4) {  // pair: value in [-3, 4] (ties are frequent), index in [0, 64); padding zero
            put_small(p, (int)(u % 8) - 3, tc.vsize, tc.vfloat);
            const int32_t idx = (int32_t)((u >> 8) & 63);
            std::memcpy(p + (tc.vsize == 8 ? 8 : 4), &idx, 4);
        } else if (tc.kind == 5) {  // complex: small integer parts, so every sum and product is exact
            put_small(p, (int)(u % 8) - 3, tc.vsize, true);
            put_small(p + tc.vsize, (int)((u >> 8) % 8) - 3, tc.vsize, true);
        } else if (tc.kind == 1) {  // small integers in [-3, 4], zeros included: every sum/product is exact
            const float f = (float)((int)(u % 8) - 3);
            std::memcpy(p, &f, 4);
        } else if (tc.kind == 2) {
            const double d = (double)((int)(u % 8) - 3);
            std::memcpy(p, &d, 8);
        } else if (tc.kind == 3) {
            p[0] = (char)((u >> 7) & 1);
        } else if ((u >> 61) == 0) {  // 1/8 zeros so the logical ops see both truth values
            std::memset(p, 0, tsize);
        } else {
            std::memcpy(p, &u, tsize);
        }
    }
}

void user_op(void*, void*, int*, MPI_Datatype*) {}

// host twins of the test launchers in tests/userop/halfadd_op.hip (MPI's own collectives run these)
void host_isum(void* in, void* inout, int* len, MPI_Datatype*) {
    const uint32_t* a = (const uint32_t*)in;
    uint32_t* b = (uint32_t*)inout;
    for (int i = 0; i < *len; ++i) b[i] = a[i] + b[i];
}
void host_mix3(void* in, void* inout, int* len, MPI_Datatype*) {
    const uint32_t* a = (const uint32_t*)in;
    uint32_t* b = (uint32_t*)inout;
    for (int i = 0; i < *len; ++i) b[i] = a[i] * 3u + b[i];
}

// Complex results compared by value: the parts are exact small integers, but a zero part's sign
// depends on the association (re = ac - bd can be +0 or -0), and MPI's own collective associates
// differently from the radix/batch schedule.  Everything else is compared bit for bit.
bool same(const std::vector<char>& a, const std::vector<char>& b, const TypeCase& tc) {
    if (tc.kind != 5) return a == b;
    if (a.size() != b.size()) return false;
    for (size_t off = 0; off < a.size(); off += (size_t)tc.vsize) {
        double x, y;
        if (tc.vsize == 4) {
            float fx, fy;
            std::memcpy(&fx, &a[off], 4);
            std::memcpy(&fy, &b[off], 4);
            x = fx;
            y = fy;
        } else {
            std::memcpy(&x, &a[off], 8);
            std::memcpy(&y, &b[off], 8);
        }
        if (!(x == y)) return false;
    }
    return true;
}

}  // namespace

int main(int argc, char** argv) {
    setenv("HSA_ENABLE_IPC_MODE_LEGACY", "0", 0);  // dmabuf IPC for RCCL, before any HIP call (api.cpp)
    MPI_Init(&argc, &argv);
    MPI_Comm_set_errhandler(MPI_COMM_WORLD, MPI_ERRORS_RETURN);
    int rank, n;
    MPI_Comm_rank(MPI_COMM_WORLD, &rank);
    MPI_Comm_size(MPI_COMM_WORLD, &n);
    const TypeCase types[] = {
        {MPI_CHAR, "MPI_CHAR", 0}, {MPI_SIGNED_CHAR, "MPI_SIGNED_CHAR", 0},
        {MPI_UNSIGNED_CHAR, "MPI_UNSIGNED_CHAR", 0}, {MPI_SHORT, "MPI_SHORT", 0},
        {MPI_UNSIGNED_SHORT, "MPI_UNSIGNED_SHORT", 0}, {MPI_INT, "MPI_INT", 0}, {MPI_UNSIGNED, "MPI_UNSIGNED", 0},
        {MPI_LONG, "MPI_LONG", 0}, {MPI_UNSIGNED_LONG, "MPI_UNSIGNED_LONG", 0}, {MPI_LONG_LONG, "MPI_LONG_LONG", 0},
        {MPI_UNSIGNED_LONG_LONG, "MPI_UNSIGNED_LONG_LONG", 0}, {MPI_INT8_T, "MPI_INT8_T", 0},
        {MPI_UINT8_T, "MPI_UINT8_T", 0}, {MPI_INT16_T, "MPI_INT16_T", 0}, {MPI_UINT16_T, "MPI_UINT16_T", 0},
        {MPI_INT32_T, "MPI_INT32_T", 0}, {MPI_UINT32_T, "MPI_UINT32_T", 0}, {MPI_INT64_T, "MPI_INT64_T", 0},
        {MPI_UINT64_T, "MPI_UINT64_T", 0}, {MPI_FLOAT, "MPI_FLOAT", 1}, {MPI_DOUBLE, "MPI_DOUBLE", 2},
        {MPI_BYTE, "MPI_BYTE", 0}, {MPI_C_BOOL, "MPI_C_BOOL", 3},
        {MPI_FLOAT_INT, "MPI_FLOAT_INT", 4, 4, true}, {MPI_DOUBLE_INT, "MPI_DOUBLE_INT", 4, 8, true},
        {MPI_LONG_INT, "MPI_LONG_INT", 4, 8, false}, {MPI_2INT, "MPI_2INT", 4, 4, false},
        {MPI_SHORT_INT, "MPI_SHORT_INT", 4, 2, false}, {MPI_C_FLOAT_COMPLEX, "MPI_C_FLOAT_COMPLEX", 5, 4, true},
        {MPI_C_COMPLEX, "MPI_C_COMPLEX", 5, 4, true}, {MPI_C_DOUBLE_COMPLEX, "MPI_C_DOUBLE_COMPLEX", 5, 8, true}};
    const struct {
        MPI_Op op;
        const char* name;
    } ops[] = {{MPI_SUM, "SUM"},   {MPI_PROD, "PROD"}, {MPI_MAX, "MAX"},   {MPI_MIN, "MIN"},  {MPI_LAND, "LAND"},
               {MPI_LOR, "LOR"},   {MPI_LXOR, "LXOR"}, {MPI_BAND, "BAND"}, {MPI_BOR, "BOR"},  {MPI_BXOR, "BXOR"},
               {MPI_MAXLOC, "MAXLOC"}, {MPI_MINLOC, "MINLOC"}};
    const int per = 37, count = per * n;
    int pairs = 0, supported = 0, bad = 0;
    std::string failures;
    auto fail = [&](const std::string& what) {
        ++bad;
        if (failures.size() < 600) failures += (failures.empty() ? "" : "; ") + what;
    };
    int salt = 0;
    for (const TypeCase& tc : types) {
        MPI_Aint lb = 0, ext = 0;
        MPI_Type_get_extent(tc.t, &lb, &ext);
        const int tsize = (int)ext;  // the element stride of a buffer
        for (const auto& o : ops) {
            ++pairs;
            ++salt;
            const std::string id = std::string(tc.name) + "/" + o.name;
            std::vector<char> probe_in(2 * (size_t)tsize, 0), probe_io(2 * (size_t)tsize, 0);
            const bool mpich_ok = MPI_Reduce_local(probe_in.data(), probe_io.data(), 1, tc.t, o.op) == MPI_SUCCESS;
            std::vector<char> send, recv((size_t)count * tsize), lib((size_t)count * tsize);
            fill(send, count, tc, tsize, rank, salt);
            // allreduce (k=2, b=2: a two-level geometry at 4 ranks) vs MPI_Allreduce
            const int rc = all_reduce_radix_batch(send.data(), recv.data(), count, tc.t, o.op, MPI_COMM_WORLD, 2,
                                                  n % 2 ? 1 : 2);
            if (!mpich_ok) {
                if (rc == MPI_SUCCESS) fail(id + " accepted, MPICH rejects it");
                continue;
            }
            ++supported;
            MPI_Allreduce(send.data(), lib.data(), count, tc.t, o.op, MPI_COMM_WORLD);
            if (rc != MPI_SUCCESS) fail(id + " allreduce rc=" + std::to_string(rc));
            else if (!same(recv, lib, tc)) fail(id + " allreduce differs from MPI_Allreduce");
            // reduce-scatter (block) vs MPI_Reduce_scatter_block
            std::vector<char> rs((size_t)per * tsize), rs_lib((size_t)per * tsize);
            const int rc2 = reduce_scatter_radix_batch(send.data(), rs.data(), per, tc.t, o.op, MPI_COMM_WORLD, 2, 1);
            MPI_Reduce_scatter_block(send.data(), rs_lib.data(), per, tc.t, o.op, MPI_COMM_WORLD);
            if (rc2 != MPI_SUCCESS || !same(rs, rs_lib, tc)) fail(id + " reduce_scatter rc=" + std::to_string(rc2));
            // an MPICH baseline testing/main.cpp drives (ring, reduction at allreduce_ring.cpp:80)
            std::vector<char> ring((size_t)count * tsize);
            const int rc3 = MPICH_Allreduce_ring(send.data(), ring.data(), count, tc.t, o.op, MPI_COMM_WORLD);
            if (rc3 != MPI_SUCCESS || !same(ring, lib, tc)) fail(id + " ring rc=" + std::to_string(rc3));
        }
    }
    // what the shim must refuse with an MPI error class
    {
        std::vector<char> a(64 * n * 16, 1), r(64 * n * 16, 0);
        MPI_Op uop;
        MPI_Op_create(user_op, 1, &uop);
        if (all_reduce_radix_batch(a.data(), r.data(), 4 * n, MPI_INT, uop, MPI_COMM_WORLD, 2, 1) == MPI_SUCCESS)
            fail("user op accepted");
        MPI_Op_free(&uop);
        if (all_reduce_radix_batch(a.data(), r.data(), 4 * n, MPI_INT, MPI_MAXLOC, MPI_COMM_WORLD, 2, 1) == MPI_SUCCESS)
            fail("MPI_MAXLOC on MPI_INT accepted");
        if (all_reduce_radix_batch(a.data(), r.data(), 4 * n, MPI_LONG_DOUBLE_INT, MPI_MAXLOC, MPI_COMM_WORLD, 2, 1) ==
            MPI_SUCCESS)
            fail("MPI_LONG_DOUBLE_INT accepted");
        if (all_reduce_radix_batch(a.data(), r.data(), 4 * n, MPI_LONG_DOUBLE, MPI_SUM, MPI_COMM_WORLD, 2, 1) ==
            MPI_SUCCESS)
            fail("MPI_LONG_DOUBLE accepted");
        if (allgather_radix_batch(a.data(), 4, MPI_DOUBLE_INT, r.data(), MPI_COMM_WORLD, 2, 1) == MPI_SUCCESS)
            fail("non-contiguous allgather type accepted");
    }
    // user ops bound to their device launchers (chiara_shim_op_bind), when the test names the launchers' library:
    // a commutative wrapping add against MPI_Allreduce / MPI_Reduce_scatter_block with the same host op; a
    // non-commutative one runs the radix/batch allreduce (every rank the same bits) and is refused by
    // k-reduce-scatter-allgather with MPI_ERR_OP, as the reference refuses it; unbound again, MPI_ERR_OP
    int userop = 0;
    if (const char* so = std::getenv("CHR_SHIM_USEROP_SO")) {
        void* h = dlopen(so, RTLD_NOW | RTLD_LOCAL);
        auto isum = h ? (user_reduce_fn)dlsym(h, "chr_test_isum") : nullptr;
        auto mix3 = h ? (user_reduce_fn)dlsym(h, "chr_test_halfadd") : nullptr;
        if (!isum || !mix3) {
            fail(std::string("user-op launchers not found in ") + so);
        } else {
            MPI_Op sop, nop;
            MPI_Op_create(host_isum, 1, &sop);
            MPI_Op_create(host_mix3, 0, &nop);
            const int per = 1001, cnt = per * n;
            TypeCase ti{MPI_INT, "MPI_INT", 0};
            std::vector<char> send, r((size_t)cnt * 4), lib((size_t)cnt * 4), rs((size_t)per * 4),
                rs_lib((size_t)per * 4);
            fill(send, cnt, ti, 4, rank, 9999);
            if (chiara_shim_op_bind(sop, isum, nullptr) != MPI_SUCCESS) fail("bind commutative user op");
            if (chiara_shim_op_bind(MPI_SUM, isum, nullptr) == MPI_SUCCESS) fail("a predefined op was bound");
            int rc = all_reduce_radix_batch(send.data(), r.data(), cnt, MPI_INT, sop, MPI_COMM_WORLD, 2, n % 2 ? 1 : 2);
            MPI_Allreduce(send.data(), lib.data(), cnt, MPI_INT, sop, MPI_COMM_WORLD);
            if (rc != MPI_SUCCESS || r != lib) fail("bound user op allreduce rc=" + std::to_string(rc));
            rc = reduce_scatter_radix_batch(send.data(), rs.data(), per, MPI_INT, sop, MPI_COMM_WORLD, 2, 1);
            MPI_Reduce_scatter_block(send.data(), rs_lib.data(), per, MPI_INT, sop, MPI_COMM_WORLD);
            if (rc != MPI_SUCCESS || rs != rs_lib) fail("bound user op reduce_scatter rc=" + std::to_string(rc));
            std::vector<char> ring((size_t)cnt * 4);
            rc = MPICH_Allreduce_ring(send.data(), ring.data(), cnt, MPI_INT, sop, MPI_COMM_WORLD);
            if (rc != MPI_SUCCESS || ring != lib) fail("bound user op ring rc=" + std::to_string(rc));
            if (chiara_shim_op_bind(nop, mix3, nullptr) != MPI_SUCCESS) fail("bind non-commutative user op");
            rc = all_reduce_radix_batch(send.data(), r.data(), cnt, MPI_INT, nop, MPI_COMM_WORLD, 2, n % 2 ? 1 : 2);
            std::vector<char> all((size_t)cnt * 4 * n);
            MPI_Allgather(r.data(), cnt * 4, MPI_BYTE, all.data(), cnt * 4, MPI_BYTE, MPI_COMM_WORLD);
            bool same_all = true;
            for (int q = 1; q < n; ++q) same_all &= std::memcmp(all.data(), all.data() + (size_t)q * cnt * 4, cnt * 4) == 0;
            if (rc != MPI_SUCCESS || !same_all) fail("non-commutative bound op allreduce rc=" + std::to_string(rc));
            rc = MPICH_Allreduce_k_reduce_scatter_allgather(send.data(), r.data(), cnt, MPI_INT, nop, MPI_COMM_WORLD,
                                                            2, 0);
            if (rc != MPI_ERR_OP) fail("k_reduce_scatter_allgather with a non-commutative op rc=" + std::to_string(rc));
            if (chiara_shim_op_unbind(sop) != MPI_SUCCESS || chiara_shim_op_unbind(nop) != MPI_SUCCESS)
                fail("unbind");
            rc = all_reduce_radix_batch(send.data(), r.data(), cnt, MPI_INT, sop, MPI_COMM_WORLD, 2, 1);
            if (rc != MPI_ERR_OP) fail("unbound user op rc=" + std::to_string(rc));
            MPI_Op_free(&sop);
            MPI_Op_free(&nop);
            userop = 1;
        }
    }
    // allgather moves any contiguous type as bytes (the reference sizes it with MPI_Type_size)
    {
        MPI_Datatype tri;
        MPI_Type_contiguous(3, MPI_SHORT, &tri);
        MPI_Type_commit(&tri);
        const int sc = 11;
        std::vector<char> s((size_t)sc * 6), g((size_t)sc * 6 * n), lib((size_t)sc * 6 * n);
        for (size_t i = 0; i < s.size(); ++i) s[i] = (char)mix(((uint64_t)rank << 32) ^ i);
        const int rc = allgather_radix_batch(s.data(), sc, tri, g.data(), MPI_COMM_WORLD, 2, 1);
        MPI_Allgather(s.data(), sc, tri, lib.data(), sc, tri, MPI_COMM_WORLD);
        if (rc != MPI_SUCCESS || g != lib) fail("allgather of a contiguous derived type");
        MPI_Type_free(&tri);
    }
    int all_bad = 0;
    MPI_Allreduce(&bad, &all_bad, 1, MPI_INT, MPI_SUM, MPI_COMM_WORLD);
    if (rank == 0)
        std::printf("{\"pairs\": %d, \"supported_by_mpich\": %d, \"failures\": %d, \"userop\": %d, \"first\": \"%s\"}\n",
                    pairs, supported, all_bad, userop, failures.c_str());
    MPI_Finalize();
    return all_bad ? 1 : 0;
}
