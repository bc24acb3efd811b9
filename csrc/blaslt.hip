// Thin hipBLASLt binding for the plain GEMMs of the model (SURVEY 2.8 K9 library path).
//
// Why a direct binding instead of torch.matmul: (1) the weight-gradient GEMM accumulates in
// place into the stage's fp32 main_grad (bf16 A/B, fp32 C = D, beta = 1), so no bf16 dW tensor
// and no separate accumulate pass exist; (2) bias, bias+GELU (saving the pre-activation as the
// AUX output), dGELU+bias-grad and bias-grad-of-A epilogues fold the pointwise work and the bias
// reductions into the GEMM.  Row-major callers map to column-major hipBLASLt by swapping
// operands (see trustworthy_dl/ops/blaslt.py).  Descriptors + the heuristic's best algorithm are
// cached per problem signature; launches go to the caller's stream, so they are graph-capturable.
#include <hip/hip_runtime.h>
#include <hipblaslt/hipblaslt.h>

#include <cstdint>
#include <cstring>
#include <map>
#include <mutex>
#include <tuple>
#include <vector>

#define TDL_API extern "C" __attribute__((visibility("default")))

namespace {

hipDataType dtype_of(int code) {
    switch (code) {
        case 1: return HIP_R_16BF;
        case 2: return HIP_R_16F;
        default: return HIP_R_32F;
    }
}

struct Key {
    int opA, opB, m, n, k, lda, ldb, ldc, ldd, tA, tB, tC, tD, epi, bias_t, ld_aux, dev;
    bool operator<(const Key& o) const {
        return std::memcmp(this, &o, sizeof(Key)) < 0;
    }
};

struct Plan {
    hipblasLtMatmulDesc_t desc = nullptr;
    hipblasLtMatrixLayout_t a = nullptr, b = nullptr, c = nullptr, d = nullptr;
    hipblasLtMatmulAlgo_t algo;
    size_t ws_needed = 0;
    bool ok = false;
};

std::mutex g_mu;
std::map<int, hipblasLtHandle_t> g_handles;
std::map<Key, Plan> g_plans;

hipblasLtHandle_t handle_for(int dev) {
    auto it = g_handles.find(dev);
    if (it != g_handles.end()) return it->second;
    hipblasLtHandle_t h = nullptr;
    if (hipblasLtCreate(&h) != HIPBLAS_STATUS_SUCCESS) return nullptr;
    g_handles[dev] = h;
    return h;
}

}  // namespace

// Return codes: 0 ok, 1 handle failure, 2 no algorithm for this configuration, 3 matmul failure,
// 4 workspace too small.
TDL_API int tdl_blaslt_gemm(int opA, int opB, int m, int n, int k, float alpha, const void* A, int lda, int tA,
                            const void* B, int ldb, int tB, float beta, const void* C, int ldc, int tC, void* D, int ldd,
                            int tD, int epilogue, const void* bias, int bias_t, void* aux, int ld_aux, void* ws,
                            int64_t ws_size, hipStream_t stream) {
    int dev = 0;
    hipGetDevice(&dev);
    Key key{opA, opB, m, n, k, lda, ldb, ldc, ldd, tA, tB, tC, tD, epilogue, bias_t, ld_aux, dev};
    Plan* plan = nullptr;
    hipblasLtHandle_t h = nullptr;
    {
        std::lock_guard<std::mutex> lk(g_mu);
        h = handle_for(dev);
        if (!h) return 1;
        auto it = g_plans.find(key);
        if (it == g_plans.end()) {
            Plan p;
            hipblasLtMatmulDescCreate(&p.desc, HIPBLAS_COMPUTE_32F, HIP_R_32F);
            hipblasOperation_t oa = opA ? HIPBLAS_OP_T : HIPBLAS_OP_N, ob = opB ? HIPBLAS_OP_T : HIPBLAS_OP_N;
            hipblasLtMatmulDescSetAttribute(p.desc, HIPBLASLT_MATMUL_DESC_TRANSA, &oa, sizeof(oa));
            hipblasLtMatmulDescSetAttribute(p.desc, HIPBLASLT_MATMUL_DESC_TRANSB, &ob, sizeof(ob));
            hipblasLtEpilogue_t epi = (hipblasLtEpilogue_t)epilogue;
            hipblasLtMatmulDescSetAttribute(p.desc, HIPBLASLT_MATMUL_DESC_EPILOGUE, &epi, sizeof(epi));
            if (epilogue != HIPBLASLT_EPILOGUE_DEFAULT) {
                const void* dummy = bias ? bias : (const void*)0x100;
                hipblasLtMatmulDescSetAttribute(p.desc, HIPBLASLT_MATMUL_DESC_BIAS_POINTER, &dummy, sizeof(dummy));
                hipDataType bt = dtype_of(bias_t);
                hipblasLtMatmulDescSetAttribute(p.desc, HIPBLASLT_MATMUL_DESC_BIAS_DATA_TYPE, &bt, sizeof(bt));
                if (aux) {
                    int64_t ld = ld_aux;
                    hipblasLtMatmulDescSetAttribute(p.desc, HIPBLASLT_MATMUL_DESC_EPILOGUE_AUX_POINTER, &aux, sizeof(aux));
                    hipblasLtMatmulDescSetAttribute(p.desc, HIPBLASLT_MATMUL_DESC_EPILOGUE_AUX_LD, &ld, sizeof(ld));
                }
            }
            const int rowsA = opA ? k : m, colsA = opA ? m : k;
            const int rowsB = opB ? n : k, colsB = opB ? k : n;
            hipblasLtMatrixLayoutCreate(&p.a, dtype_of(tA), rowsA, colsA, lda);
            hipblasLtMatrixLayoutCreate(&p.b, dtype_of(tB), rowsB, colsB, ldb);
            hipblasLtMatrixLayoutCreate(&p.c, dtype_of(tC), m, n, ldc);
            hipblasLtMatrixLayoutCreate(&p.d, dtype_of(tD), m, n, ldd);
            hipblasLtMatmulPreference_t pref;
            hipblasLtMatmulPreferenceCreate(&pref);
            uint64_t max_ws = (uint64_t)ws_size;
            hipblasLtMatmulPreferenceSetAttribute(pref, HIPBLASLT_MATMUL_PREF_MAX_WORKSPACE_BYTES, &max_ws, sizeof(max_ws));
            hipblasLtMatmulHeuristicResult_t res[8];
            int got = 0;
            hipblasStatus_t st = hipblasLtMatmulAlgoGetHeuristic(h, p.desc, p.a, p.b, p.c, p.d, pref, 8, res, &got);
            hipblasLtMatmulPreferenceDestroy(pref);
            if (st == HIPBLAS_STATUS_SUCCESS && got > 0) {
                p.algo = res[0].algo;
                p.ws_needed = res[0].workspaceSize;
                p.ok = true;
            }
            it = g_plans.emplace(key, p).first;
        }
        plan = &it->second;
    }
    if (!plan->ok) return 2;
    if (plan->ws_needed > (size_t)ws_size) return 4;
    if (epilogue != HIPBLASLT_EPILOGUE_DEFAULT) {
        // per-call pointers (the plan is shared by every call with the same signature)
        hipblasLtMatmulDescSetAttribute(plan->desc, HIPBLASLT_MATMUL_DESC_BIAS_POINTER, &bias, sizeof(bias));
        if (aux) hipblasLtMatmulDescSetAttribute(plan->desc, HIPBLASLT_MATMUL_DESC_EPILOGUE_AUX_POINTER, &aux, sizeof(aux));
    }
    hipblasStatus_t st = hipblasLtMatmul(h, plan->desc, &alpha, A, plan->a, B, plan->b, &beta, C, plan->c, D, plan->d,
                                         &plan->algo, ws, (size_t)ws_size, stream);
    return st == HIPBLAS_STATUS_SUCCESS ? 0 : 3;
}

TDL_API int tdl_blaslt_plan_count() {
    std::lock_guard<std::mutex> lk(g_mu);
    return (int)g_plans.size();
}
