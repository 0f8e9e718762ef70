// mock_icicle.cpp -- stands in for ICICLE core in tests (ICICLE is not in this image).
//
// Defines the icicle::register_* entry points the backend libraries bind to at dlopen time
// (same signatures as midnight-bls12-381-cuda_amd/csrc/icicle_api.hpp, i.e. the reference's
// icicle_backend_api.cuh), loads the three backend libraries the way ICICLE's backend loader
// does, and prints what was registered under which device type.
//   mock_icicle <lib/icicle dir>          registrations only (no GPU needed)
//   mock_icicle <lib/icicle dir> --run    also drives every registered op on the GPU through
//                                         the registered DeviceAPI and checks each result
//                                         byte-for-byte against the direct C ABI call
// Test infrastructure only (tests/test_icicle_backend.py).
#include <dlfcn.h>
#include <stdio.h>
#include <string.h>

#include <map>
#include <string>
#include <vector>

#include "icicle_api.hpp"

namespace mock {
using icicle::affine_t;
using icicle::Device;
using icicle::DeviceAPI;
using icicle::DeviceProperties;
using icicle::eCopyDirection;
using icicle::eIcicleError;
using icicle::icicleStreamHandle;
using icicle::MSMConfig;
using icicle::MsmImpl;
using icicle::MsmPreComputeImpl;
using icicle::NTTConfig;
using icicle::NTTDir;
using icicle::NttGetRouFromDomainImpl;
using icicle::NttImpl;
using icicle::NTTInitDomainConfig;
using icicle::NttInitDomainImpl;
using icicle::NttReleaseDomainImpl;
using icicle::projective_t;
using icicle::scalar_t;
using icicle::scalarVectorOpImpl;
using icicle::VecOpsConfig;
using icicle::VectorReduceOpImpl;

// ---- the mock registry ------------------------------------------------------------------
static std::map<std::string, std::vector<std::string>>& regs() {
    static std::map<std::string, std::vector<std::string>> m;
    return m;
}
// function-local statics: the backend libraries linked into this executable register from
// their own static initialisers, which run before this executable's globals are constructed
#define MOCK_MAP(NAME, TYPE)                                   \
    static std::map<std::string, TYPE>& NAME() {               \
        static std::map<std::string, TYPE> m;                  \
        return m;                                              \
    }
MOCK_MAP(g_ntt, NttImpl)
MOCK_MAP(g_ntt_init, NttInitDomainImpl)
MOCK_MAP(g_ntt_rel, NttReleaseDomainImpl)
MOCK_MAP(g_rou, NttGetRouFromDomainImpl)
MOCK_MAP(g_vadd, scalarVectorOpImpl)
MOCK_MAP(g_vsub, scalarVectorOpImpl)
MOCK_MAP(g_vmul, scalarVectorOpImpl)
MOCK_MAP(g_smul, scalarVectorOpImpl)
MOCK_MAP(g_sadd, scalarVectorOpImpl)
MOCK_MAP(g_vsum, VectorReduceOpImpl)
MOCK_MAP(g_msm, MsmImpl)
MOCK_MAP(g_msm_pre, MsmPreComputeImpl)
MOCK_MAP(g_dev, std::shared_ptr<DeviceAPI>)
}  // namespace mock

#define MOCK_REG(NAME, MAP, TYPE)                                  \
    void NAME(const std::string& deviceType, TYPE impl) {          \
        mock::regs()[#NAME].push_back(deviceType);                 \
        mock::MAP()[deviceType] = impl;                            \
    }
namespace icicle {
MOCK_REG(register_ntt, g_ntt, NttImpl)
MOCK_REG(register_ntt_init_domain, g_ntt_init, NttInitDomainImpl)
MOCK_REG(register_ntt_release_domain, g_ntt_rel, NttReleaseDomainImpl)
MOCK_REG(register_ntt_get_rou_from_domain, g_rou, NttGetRouFromDomainImpl)
MOCK_REG(register_vector_add, g_vadd, scalarVectorOpImpl)
MOCK_REG(register_vector_sub, g_vsub, scalarVectorOpImpl)
MOCK_REG(register_vector_mul, g_vmul, scalarVectorOpImpl)
MOCK_REG(register_scalar_mul_vec, g_smul, scalarVectorOpImpl)
MOCK_REG(register_scalar_add_vec, g_sadd, scalarVectorOpImpl)
MOCK_REG(register_vector_sum, g_vsum, VectorReduceOpImpl)
MOCK_REG(register_msm, g_msm, MsmImpl)
MOCK_REG(register_msm_precompute_bases, g_msm_pre, MsmPreComputeImpl)
void register_deviceAPI(const std::string& deviceType, std::shared_ptr<DeviceAPI> api) {
    mock::regs()["register_deviceAPI"].push_back(deviceType);
    mock::g_dev()[deviceType] = api;
}
}  // namespace icicle

// ---- GPU drive (--run) -------------------------------------------------------------------
namespace mock {
static int failures = 0;
#define CHECK(cond, what)                                   \
    do {                                                    \
        if (!(cond)) {                                      \
            fprintf(stderr, "FAIL: %s\n", what);            \
            ++failures;                                     \
        }                                                   \
    } while (0)

template <class F>
static F sym(const char* name) {
    F f = reinterpret_cast<F>(dlsym(RTLD_DEFAULT, name));
    if (!f) fprintf(stderr, "missing symbol %s\n", name);
    return f;
}

static int run_gpu(const char* dev_type) {
    DeviceAPI* api = g_dev().at(dev_type).get();
    // ICICLE's Device is {char type[32]; int id} (include/icicle/device.h:55-57): build it the
    // way ICICLE's constructor does, so a backend reading `id` at the wrong offset is caught
    auto make_dev = [](const char* type, int id) { return icicle::make_device(type, id); };
    Device dev = make_dev(dev_type, 0);
    int count = 0;
    CHECK(api->get_device_count(count) == eIcicleError::SUCCESS && count >= 1, "get_device_count");
    // an id past the last device must be rejected, not silently mapped to device 0
    CHECK(api->set_device(make_dev(dev_type, count)) == eIcicleError::INVALID_DEVICE, "set_device(id = count) rejected");
    CHECK(api->set_device(make_dev(dev_type, -1)) == eIcicleError::INVALID_DEVICE, "set_device(id = -1) rejected");
    CHECK(api->set_device(dev) == eIcicleError::SUCCESS, "set_device");
    {  // HostToHost (device_api.h:44) is a host memcpy, not a device-to-device copy
        uint8_t src[64], dst[64];
        for (int i = 0; i < 64; ++i) src[i] = (uint8_t)(3 * i + 1), dst[i] = 0;
        CHECK(api->copy(dst, src, 64, eCopyDirection::HostToHost) == eIcicleError::SUCCESS && memcmp(dst, src, 64) == 0,
              "copy HostToHost");
    }
    icicleStreamHandle st = nullptr;
    CHECK(api->create_stream(&st) == eIcicleError::SUCCESS && st, "create_stream");

    auto gen_scalars = sym<::eIcicleError (*)(mbls_fr_t*, uint64_t, size_t, bool, void*)>("mbls_gen_scalars");
    auto gen_g1 = sym<::eIcicleError (*)(mbls_g1_affine_t*, uint64_t, size_t, void*)>("mbls_gen_g1_bases");
    auto gen_g2 = sym<::eIcicleError (*)(mbls_g2_affine_t*, uint64_t, size_t, void*)>("mbls_gen_g2_bases");
    auto def_msm = sym<::MSMConfig (*)()>("mbls_default_msm_config");
    auto def_ntt = sym<::NTTConfig (*)()>("mbls_default_ntt_config");
    auto def_vec = sym<::VecOpsConfig (*)()>("mbls_default_vec_ops_config");
    auto g2_via_registry = sym<::eIcicleError (*)(const char*, const mbls_fr_t*, const mbls_g2_affine_t*, int,
                                                  const ::MSMConfig*, mbls_g2_projective_t*)>(
        "mbls_icicle_g2_msm_via_registry");
    if (!gen_scalars || !gen_g1 || !gen_g2 || !def_msm || !def_ntt || !def_vec || !g2_via_registry) return 1;

    const size_t n = 4096;
    void *s = nullptr, *b1 = nullptr, *b2 = nullptr, *v = nullptr, *w = nullptr, *o1 = nullptr, *o2 = nullptr;
    CHECK(api->allocate_memory(&s, n * 32) == eIcicleError::SUCCESS, "allocate scalars");
    CHECK(api->allocate_memory(&b1, n * 96) == eIcicleError::SUCCESS, "allocate g1 bases");
    CHECK(api->allocate_memory(&b2, n * 192) == eIcicleError::SUCCESS, "allocate g2 bases");
    CHECK(api->allocate_memory_async(&v, n * 32, st) == eIcicleError::SUCCESS, "allocate_async v");
    CHECK(api->allocate_memory(&w, n * 32) == eIcicleError::SUCCESS, "allocate w");
    CHECK(api->allocate_memory(&o1, n * 32) == eIcicleError::SUCCESS, "allocate o1");
    CHECK(api->allocate_memory(&o2, n * 32) == eIcicleError::SUCCESS, "allocate o2");
    CHECK(api->memset_async(o1, 0, n * 32, st) == eIcicleError::SUCCESS, "memset_async");
    gen_scalars((mbls_fr_t*)s, 11, n, true, st);
    gen_scalars((mbls_fr_t*)v, 12, n, true, st);
    gen_scalars((mbls_fr_t*)w, 13, n, true, st);
    gen_g1((mbls_g1_affine_t*)b1, 14, n, st);
    gen_g2((mbls_g2_affine_t*)b2, 15, n, st);
    CHECK(api->synchronize(st) == eIcicleError::SUCCESS, "synchronize");

    // G1 MSM: registered impl vs direct ICICLE-semantics entry point
    ::MSMConfig mc = def_msm();
    mc.stream = st;
    mc.are_scalars_on_device = mc.are_points_on_device = true;
    mc.are_scalars_montgomery_form = true;
    mc.are_points_montgomery_form = true;  // mbls_gen_* bases are Montgomery (a second conversion
                                           // would leave the curve, and sums of off-curve points
                                           // depend on the addition order)
    mc.are_results_on_device = false;
    std::vector<uint8_t> r_reg(288), r_dir(288);
    const MSMConfig& imc = *reinterpret_cast<const MSMConfig*>(&mc);
    CHECK(g_msm().at(dev_type)(dev, (const scalar_t*)s, (const affine_t*)b1, (int)n, imc, (projective_t*)r_reg.data()) ==
              eIcicleError::SUCCESS,
          "registered g1 msm");
    CHECK(bls12_381_icicle_g1_msm((const mbls_fr_t*)s, (const mbls_g1_affine_t*)b1, (int)n, &mc,
                                  (mbls_g1_projective_t*)r_dir.data()) == MBLS_SUCCESS,
          "direct g1 msm");
    CHECK(memcmp(r_reg.data(), r_dir.data(), 144) == 0, "g1 msm result equality");
    // G2 MSM through the curve backend's own registry
    CHECK(g2_via_registry(dev_type, (const mbls_fr_t*)s, (const mbls_g2_affine_t*)b2, (int)n, &mc,
                          (mbls_g2_projective_t*)r_reg.data()) == MBLS_SUCCESS,
          "registered g2 msm");
    CHECK(bls12_381_icicle_g2_msm((const mbls_fr_t*)s, (const mbls_g2_affine_t*)b2, (int)n, &mc,
                                  (mbls_g2_projective_t*)r_dir.data()) == MBLS_SUCCESS,
          "direct g2 msm");
    CHECK(memcmp(r_reg.data(), r_dir.data(), 288) == 0, "g2 msm result equality");

    // NTT: init domain through the registry, forward transform vs direct
    scalar_t root;
    memset(&root, 0, sizeof(root));
    ::NTTInitDomainConfig ic{st, false, nullptr};
    CHECK(g_rou().at(dev_type)(dev, 12, &root) == eIcicleError::INVALID_ARGUMENT, "rou before init rejected");
    {  // initialise with the canonical 2^32-th root of unity, Montgomery (bls12_381_constants.h:127-130)
        mbls_fr_t w32 = {{0xb9b58d8c5f0e466aULL, 0x5b1b4c801819d7ecULL, 0x0af53ae352a31e64ULL, 0x5bf3adda19e9b27bULL}};
        memcpy(&root, &w32, 32);
    }
    CHECK(g_ntt_init().at(dev_type)(dev, root, *reinterpret_cast<const NTTInitDomainConfig*>(&ic)) ==
              eIcicleError::SUCCESS,
          "registered ntt init domain");
    scalar_t w12, w12d;
    CHECK(g_rou().at(dev_type)(dev, 12, &w12) == eIcicleError::SUCCESS, "registered rou");
    CHECK(bls12_381_ntt_get_rou_from_domain(12, (mbls_fr_t*)&w12d) == MBLS_SUCCESS && memcmp(&w12, &w12d, 32) == 0,
          "rou equality");
    ::NTTConfig nc = def_ntt();
    nc.stream = st;
    nc.are_inputs_on_device = nc.are_outputs_on_device = true;
    CHECK(g_ntt().at(dev_type)(dev, (const scalar_t*)v, (int)n, NTTDir::kForward,
                             *reinterpret_cast<const NTTConfig<scalar_t>*>(&nc), (scalar_t*)o1) == eIcicleError::SUCCESS,
          "registered ntt");
    CHECK(bls12_381_ntt_cuda((const mbls_fr_t*)v, (int)n, MBLS_NTT_FORWARD, &nc, (mbls_fr_t*)o2) == MBLS_SUCCESS,
          "direct ntt");
    std::vector<uint8_t> h1(n * 32), h2(n * 32);
    api->copy(h1.data(), o1, n * 32, eCopyDirection::DeviceToHost);
    api->copy(h2.data(), o2, n * 32, eCopyDirection::DeviceToHost);
    CHECK(h1 == h2, "ntt result equality");

    // vector ops (device operands) and vector_sum (host operand, staged by the backend)
    ::VecOpsConfig vc = def_vec();
    vc.stream = st;
    vc.is_a_on_device = vc.is_b_on_device = vc.is_result_on_device = true;
    const VecOpsConfig& ivc = *reinterpret_cast<const VecOpsConfig*>(&vc);
    struct {
        const char* name;
        std::map<std::string, scalarVectorOpImpl>& (*reg)();
        ::eIcicleError (*direct)(const mbls_fr_t*, const mbls_fr_t*, size_t, const ::VecOpsConfig*, mbls_fr_t*);
        size_t na;
    } ops[] = {{"vector_add", g_vadd, bls12_381_vector_add, n},
               {"vector_sub", g_vsub, bls12_381_vector_sub, n},
               {"vector_mul", g_vmul, bls12_381_vector_mul, n},
               {"scalar_mul_vec", g_smul, bls12_381_scalar_mul_vec, 1},
               {"scalar_add_vec", g_sadd, bls12_381_scalar_add_vec, 1}};
    for (auto& op : ops) {
        CHECK(op.reg().at(dev_type)(dev, (const scalar_t*)v, (const scalar_t*)w, n, ivc, (scalar_t*)o1) ==
                  eIcicleError::SUCCESS,
              op.name);
        CHECK(op.direct((const mbls_fr_t*)v, (const mbls_fr_t*)w, n, &vc, (mbls_fr_t*)o2) == MBLS_SUCCESS, op.name);
        api->synchronize(st);
        api->copy(h1.data(), o1, n * 32, eCopyDirection::DeviceToHost);
        api->copy(h2.data(), o2, n * 32, eCopyDirection::DeviceToHost);
        CHECK(h1 == h2, op.name);
    }
    ::VecOpsConfig sc = vc;
    sc.is_a_on_device = false;
    sc.is_result_on_device = false;
    sc.is_async = false;
    std::vector<uint8_t> host_v(n * 32), sum_reg(32), sum_dir(32);
    api->copy(host_v.data(), v, n * 32, eCopyDirection::DeviceToHost);
    CHECK(g_vsum().at(dev_type)(dev, (const scalar_t*)host_v.data(), n, *reinterpret_cast<const VecOpsConfig*>(&sc),
                              (scalar_t*)sum_reg.data()) == eIcicleError::SUCCESS,
          "registered vector_sum");
    ::VecOpsConfig dc = vc;
    dc.is_result_on_device = false;
    dc.is_async = false;
    CHECK(vec_sum_cuda((mbls_fr_t*)sum_dir.data(), (const mbls_fr_t*)v, (int)n, &dc) == MBLS_SUCCESS, "direct vec_sum");
    CHECK(sum_reg == sum_dir, "vector_sum equality");

    scalar_t phantom;
    CHECK(g_ntt_rel().at(dev_type)(dev, phantom) == eIcicleError::SUCCESS, "registered release domain");
    CHECK(api->free_memory_async(v, st) == eIcicleError::SUCCESS, "free_async");
    for (void* p : {s, b1, b2, w, o1, o2}) CHECK(api->free_memory(p) == eIcicleError::SUCCESS, "free");
    CHECK(api->synchronize(st) == eIcicleError::SUCCESS, "final synchronize");
    CHECK(api->destroy_stream(st) == eIcicleError::SUCCESS, "destroy_stream");
    size_t total = 0, freeb = 0;
    CHECK(api->get_available_memory(total, freeb) == eIcicleError::SUCCESS && total >= freeb && total > 0, "meminfo");
    DeviceProperties props;
    CHECK(api->get_device_properties(props) == eIcicleError::SUCCESS && !props.using_host_memory, "properties");
    return failures;
}
}  // namespace mock

int main(int argc, char** argv) {
    if (argc < 2) {
        fprintf(stderr, "usage: %s <lib/icicle dir> [--run]\n", argv[0]);
        return 2;
    }
    const std::string dir = argv[1];
    for (const char* name : {"libicicle_backend_cuda_device.so", "libicicle_backend_cuda_field_bls12_381.so",
                             "libicicle_backend_cuda_curve_bls12_381.so"}) {
        const std::string path = dir + "/" + name;
        if (!dlopen(path.c_str(), RTLD_NOW | RTLD_GLOBAL)) {
            fprintf(stderr, "dlopen %s: %s\n", path.c_str(), dlerror());
            return 3;
        }
    }
    // registrations as JSON: {"register_x": ["CUDA"], ...}
    printf("{");
    bool first = true;
    for (auto& kv : mock::regs()) {
        printf("%s\"%s\": [", first ? "" : ", ", kv.first.c_str());
        for (size_t i = 0; i < kv.second.size(); ++i) printf("%s\"%s\"", i ? ", " : "", kv.second[i].c_str());
        printf("]");
        first = false;
    }
    auto g2 = icicle::get_g2_msm_backend(icicle::backend_device_type());
    auto g2p = icicle::get_g2_precompute_backend(icicle::backend_device_type());
    printf("%s\"register_g2_msm\": [%s], \"register_g2_msm_precompute_bases\": [%s]}\n", first ? "" : ", ",
           g2 ? "\"CUDA\"" : "", g2p ? "\"CUDA\"" : "");
    fflush(stdout);
    if (argc > 2 && strcmp(argv[2], "--run") == 0) {
        const int f = mock::run_gpu(icicle::backend_device_type());
        printf(f ? "gpu run: %d failures\n" : "gpu run ok\n", f);
        return f ? 1 : 0;
    }
    return 0;
}
