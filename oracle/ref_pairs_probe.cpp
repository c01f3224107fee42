// ref_pairs_probe.cpp -- TEST INFRASTRUCTURE ONLY, container-only.
//
// Asks MPICH 3.3.2 itself (the library behind every MPI_Reduce_local of the reference,
// Fugaku_experiments/Allreduce/all_reduce_radix_batch.cpp:332, :364, :446, :529) what it does with
// the pair types (MAXLOC / MINLOC) and the C complex types, so that the oracle's restatement of
// those element semantics is pinned by MPICH's own outputs (tests/golden/gen_pairs.py writes them
// as fixtures into tests/golden/pairs_reduce_local.npz).
//
//   ref_pairs_probe table                      -> JSON: size / extent per type, and which of the
//                                                 12 predefined ops MPI_Reduce_local accepts for it
//   ref_pairs_probe reduce TYPE OP N in inout out -> out = MPI_Reduce_local(in, inout) on N elements
//                                                 (raw bytes at the type's extent); TYPE also f32 / f64
//                                                 (MPI_FLOAT / MPI_DOUBLE, for the NaN-payload fixture,
//                                                 tests/golden/gen_nan_payloads.py)
#include <mpi.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

struct Named {
    const char* name;
    MPI_Datatype t;
};

static std::vector<Named> types() {
    return {{"fi", MPI_FLOAT_INT},         {"di", MPI_DOUBLE_INT},       {"li", MPI_LONG_INT},
            {"2i", MPI_2INT},              {"si", MPI_SHORT_INT},        {"cf", MPI_C_FLOAT_COMPLEX},
            {"cd", MPI_C_DOUBLE_COMPLEX}, {"ldi", MPI_LONG_DOUBLE_INT}, {"cld", MPI_C_LONG_DOUBLE_COMPLEX}};
}

static std::vector<std::pair<const char*, MPI_Op>> ops() {
    return {{"sum", MPI_SUM},   {"prod", MPI_PROD}, {"max", MPI_MAX},   {"min", MPI_MIN},
            {"land", MPI_LAND}, {"lor", MPI_LOR},   {"lxor", MPI_LXOR}, {"band", MPI_BAND},
            {"bor", MPI_BOR},   {"bxor", MPI_BXOR}, {"maxloc", MPI_MAXLOC}, {"minloc", MPI_MINLOC}};
}

int main(int argc, char** argv) {
    MPI_Init(&argc, &argv);
    MPI_Comm_set_errhandler(MPI_COMM_WORLD, MPI_ERRORS_RETURN);
    MPI_Comm_set_errhandler(MPI_COMM_SELF, MPI_ERRORS_RETURN);
    int rc = 0;
    const std::string cmd = argc > 1 ? argv[1] : "";
    if (cmd == "table") {
        std::printf("{");
        bool first = true;
        for (const Named& t : types()) {
            int size = 0;
            MPI_Aint lb = 0, extent = 0;
            MPI_Type_size(t.t, &size);
            MPI_Type_get_extent(t.t, &lb, &extent);
            std::vector<char> a(4 * extent, 0), b(4 * extent, 0);
            std::printf("%s\"%s\": {\"size\": %d, \"extent\": %ld, \"ops\": [", first ? "" : ", ", t.name, size,
                        (long)extent);
            first = false;
            bool f2 = true;
            for (auto& o : ops()) {
                if (MPI_Reduce_local(a.data(), b.data(), 4, t.t, o.second) == MPI_SUCCESS) {
                    std::printf("%s\"%s\"", f2 ? "" : ", ", o.first);
                    f2 = false;
                }
            }
            std::printf("]}");
        }
        std::printf("}\n");
    } else if (cmd == "reduce" && argc == 8) {
        MPI_Datatype t = MPI_DATATYPE_NULL;
        std::vector<Named> all = types();
        all.push_back({"f32", MPI_FLOAT});
        all.push_back({"f64", MPI_DOUBLE});
        for (const Named& x : all)
            if (x.name == std::string(argv[2])) t = x.t;
        MPI_Op op = MPI_OP_NULL;
        for (auto& o : ops())
            if (o.first == std::string(argv[3])) op = o.second;
        const long n = std::atol(argv[4]);
        MPI_Aint lb = 0, extent = 0;
        MPI_Type_get_extent(t, &lb, &extent);
        std::vector<char> in(n * extent), io(n * extent);
        FILE* f = std::fopen(argv[5], "rb");
        rc |= f == nullptr || std::fread(in.data(), 1, in.size(), f) != in.size();
        if (f) std::fclose(f);
        f = std::fopen(argv[6], "rb");
        rc |= f == nullptr || std::fread(io.data(), 1, io.size(), f) != io.size();
        if (f) std::fclose(f);
        if (!rc) rc = MPI_Reduce_local(in.data(), io.data(), (int)n, t, op) != MPI_SUCCESS;
        f = std::fopen(argv[7], "wb");
        if (f) {
            std::fwrite(io.data(), 1, io.size(), f);
            std::fclose(f);
        }
    } else {
        std::fprintf(stderr, "usage: ref_pairs_probe table | reduce TYPE OP N in inout out\n");
        rc = 2;
    }
    MPI_Finalize();
    return rc;
}
