// pqh_forest_files.cpp -- whole-file forms of the forest builder, used by the CLI tools
// compute_nn_fast and mst_builder (csrc/tools).  Same files as the reference:
//   compute_nn_fast.c:224-225,650-651  nn_indices.ivecsl / nn_dist.fvecsl (u32 N, u32 num_nn,
//                                      rows; temp_file_to_result, fast_nn_temp_file.c:253-301)
//   fast_nn_blocks_info.c:124-172      --blocks-info-cache (blocks_info_save_file layout)
//   compute_nn_fast.c:226-230,474      --with-blocks-stat: blocks_stat.txt, "%d " per block
//   mst_builder.c:98-131               mst.tree (tree_save_file, mst.c:253-265), stats.json and
//                                      stats_num_children.json (tree_estimate_huffman_encoding,
//                                      mst.c:496-530, appended as stats.c writes them)
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "huffman.h"
#include "pq.h"
#include "pqh_internal.h"
#include "stats.h"
#include "vecs_io.h"

namespace {

struct CtxGuard {
    pqh_ctx_t* ctx = nullptr;
    ~CtxGuard() { pqh_ctx_destroy(ctx); }
};

template <typename T>
struct DevBuf {
    T* p = nullptr;
    ~DevBuf() {
        if (p) (void)hipFree(p);
    }
    int alloc(pqh_ctx* ctx, size_t count) {
        PQH_HIP(ctx, hipMalloc(&p, count * sizeof(T) + 16));
        return PQH_OK;
    }
};

std::string path_of(const char* prefix, const char* name) { return std::string(prefix) + name; }

// blocks_info_save_file / _load_file (fast_nn_blocks_info.c:124-172): field by field
bool cache_load(const char* path, int* ns, int* nb, double* overlap, std::vector<float>* st,
                std::vector<float>* en) {
    FILE* f = fopen(path, "rb");
    if (!f) return false;
    long long total = 0;
    bool ok = fread(ns, sizeof(int), 1, f) == 1 && fread(overlap, sizeof(double), 1, f) == 1 &&
              fread(nb, sizeof(int), 1, f) == 1 && fread(&total, sizeof(long long), 1, f) == 1 &&
              *ns > 0 && *ns <= 8 && *nb > 0 && *nb <= 32;
    if (ok) {
        st->assign((size_t)*ns * *nb, 0.0f);
        en->assign((size_t)*ns * *nb, 0.0f);
        for (int i = 0; ok && i < *ns; ++i) {
            int dim = 0;
            long long mask = 0;
            std::vector<float> se((size_t)2 * *nb);
            ok = fread(&dim, sizeof(int), 1, f) == 1 && fread(&mask, sizeof(long long), 1, f) == 1 &&
                 fread(se.data(), sizeof(float), se.size(), f) == se.size() && dim == *ns - 1 - i;
            std::memcpy(st->data() + (size_t)i * *nb, se.data(), sizeof(float) * *nb);
            std::memcpy(en->data() + (size_t)i * *nb, se.data() + *nb, sizeof(float) * *nb);
        }
    }
    fclose(f);
    return ok;
}

bool cache_save(const char* path, int ns, int nb, double overlap, const std::vector<float>& st,
                const std::vector<float>& en) {
    FILE* f = fopen(path, "wb");
    if (!f) return false;
    long long total = 1;
    for (int i = 0; i < ns; ++i) total *= nb;
    bool ok = fwrite(&ns, sizeof(int), 1, f) == 1 && fwrite(&overlap, sizeof(double), 1, f) == 1 &&
              fwrite(&nb, sizeof(int), 1, f) == 1 && fwrite(&total, sizeof(long long), 1, f) == 1;
    for (int i = 0; ok && i < ns; ++i) {
        const int dim = ns - 1 - i;
        long long mask = 1;
        for (int q = 0; q < dim; ++q) mask *= nb;
        ok = fwrite(&dim, sizeof(int), 1, f) == 1 && fwrite(&mask, sizeof(long long), 1, f) == 1 &&
             fwrite(st.data() + (size_t)i * nb, sizeof(float), nb, f) == (size_t)nb &&
             fwrite(en.data() + (size_t)i * nb, sizeof(float), nb, f) == (size_t)nb;
    }
    return fclose(f) == 0 && ok;
}

bool write_rows(const std::string& path, long long n, int cols, const void* data, size_t esz) {
    FILE* f = fopen(path.c_str(), "wb");
    if (!f) return false;
    save_vecs_light_meta_file(f, n, cols);
    const bool ok = fwrite(data, esz * cols, (size_t)n, f) == (size_t)n;
    return fclose(f) == 0 && ok;
}

}  // namespace

extern "C" int pqh_knn_fast_files(const char* input_fvecs, const char* out_template, int num_nn,
                                  const pqh_knn_options_t* options) {
    pqh_knn_options_t opt = {5, 3, 0.3, nullptr, 0};   // compute_nn_fast.c:164-175 defaults
    if (options) opt = *options;
    if (!input_fvecs || !out_template || num_nn <= 0) return PQH_ERR_ARG;
    long long n = 0;
    int d = 0;
    float* x = fvecs_load(input_fvecs, &n, &d);
    if (!x) return PQH_ERR_ARG;
    std::vector<float> xs(x, x + (size_t)n * d);
    free(x);
    CtxGuard g;
    int rc = pqh_ctx_create(&g.ctx, 0);
    if (rc) return rc;
    pqh_ctx* ctx = g.ctx;
    DevBuf<float> dx, dd;
    DevBuf<uint32_t> di;
    if ((rc = dx.alloc(ctx, xs.size())) || (rc = dd.alloc(ctx, (size_t)n * num_nn)) ||
        (rc = di.alloc(ctx, (size_t)n * num_nn)))
        return rc;
    PQH_HIP(ctx, hipMemcpyAsync(dx.p, xs.data(), xs.size() * 4, hipMemcpyHostToDevice, ctx->stream));
    int ns = opt.num_split, nb = opt.blocks_per_dim;
    double ov = opt.overlap;
    std::vector<float> st, en;
    // blocks info: from the cache when it loads (its geometry wins, as in the reference),
    // else computed and, with a cache path, saved (compute_nn_fast.c:633-645)
    if (!(opt.blocks_info_cache && cache_load(opt.blocks_info_cache, &ns, &nb, &ov, &st, &en))) {
        st.assign((size_t)ns * nb, 0.0f);
        en.assign((size_t)ns * nb, 0.0f);
        if ((rc = pqh_knn_blocks_info(ctx, dx.p, n, d, d, ns, nb, ov, st.data(), en.data()))) return rc;
        if (opt.blocks_info_cache && !cache_save(opt.blocks_info_cache, ns, nb, ov, st, en))
            return pqh_set_error(ctx, PQH_ERR_ARG, "cannot write %s", opt.blocks_info_cache);
    }
    long long nblocks = 1;
    for (int i = 0; i < ns; ++i) nblocks *= nb;
    std::vector<long long> sizes((size_t)nblocks);
    if ((rc = pqh_knn_fast(ctx, dx.p, n, d, d, num_nn, ns, nb, st.data(), en.data(), di.p, dd.p,
                           sizes.data())))
        return rc;
    std::vector<uint32_t> hi((size_t)n * num_nn);
    std::vector<float> hd((size_t)n * num_nn);
    PQH_HIP(ctx, hipMemcpyAsync(hi.data(), di.p, hi.size() * 4, hipMemcpyDeviceToHost, ctx->stream));
    PQH_HIP(ctx, hipMemcpyAsync(hd.data(), dd.p, hd.size() * 4, hipMemcpyDeviceToHost, ctx->stream));
    PQH_HIP(ctx, hipStreamSynchronize(ctx->stream));
    if (!write_rows(path_of(out_template, "nn_indices.ivecsl"), n, num_nn, hi.data(), 4) ||
        !write_rows(path_of(out_template, "nn_dist.fvecsl"), n, num_nn, hd.data(), 4))
        return PQH_ERR_ARG;
    if (opt.with_blocks_stat) {
        FILE* f = fopen(path_of(out_template, "blocks_stat.txt").c_str(), "w");
        if (!f) return PQH_ERR_ARG;
        for (long long b = 0; b < nblocks; ++b) fprintf(f, "%d ", (int)sizes[(size_t)b]);
        if (fclose(f) != 0) return PQH_ERR_ARG;
    }
    printf("compute_nn_fast: %lld vectors x %d dims, %lld blocks (%d splits x %d, overlap %g), "
           "%d nn\n", n, d, nblocks, ns, nb, ov, num_nn);
    return PQH_OK;
}

extern "C" int pqh_mst_files(const char* nn_template, const char* out_template, int take,
                             const char* pq_template, float penalty) {
    if (!nn_template || !out_template || take <= 0) return PQH_ERR_ARG;
    long long n = 0, n2 = 0, npq = 0;
    int num_nn = 0, num_nn2 = 0, pq_m = 0;
    byte_t* idx = load_vecs_light_filename(path_of(nn_template, "nn_indices.ivecsl").c_str(), 4,
                                           &n, &num_nn);
    byte_t* dist = load_vecs_light_filename(path_of(nn_template, "nn_dist.fvecsl").c_str(), 4,
                                            &n2, &num_nn2);
    byte_t* pq = pq_template ? load_vecs_light_filename(
                                   path_of(pq_template, "pq_indices.bvecsl").c_str(), 1, &npq, &pq_m)
                             : nullptr;
    struct Free {
        void* a[3];
        ~Free() {
            for (void* p : a) free(p);
        }
    } fr{{idx, dist, pq}};
    if (!idx || !dist || n != n2 || num_nn != num_nn2 || take > num_nn || (pq_template && (!pq || npq != n)))
        return PQH_ERR_ARG;
    CtxGuard g;
    int rc = pqh_ctx_create(&g.ctx, 0);
    if (rc) return rc;
    pqh_ctx* ctx = g.ctx;
    DevBuf<uint32_t> di;
    DevBuf<float> dd;
    DevBuf<uint8_t> dp;
    if ((rc = di.alloc(ctx, (size_t)n * num_nn)) || (rc = dd.alloc(ctx, (size_t)n * num_nn)) ||
        (pq && (rc = dp.alloc(ctx, (size_t)n * pq_m))))
        return rc;
    PQH_HIP(ctx, hipMemcpyAsync(di.p, idx, (size_t)n * num_nn * 4, hipMemcpyHostToDevice, ctx->stream));
    PQH_HIP(ctx, hipMemcpyAsync(dd.p, dist, (size_t)n * num_nn * 4, hipMemcpyHostToDevice, ctx->stream));
    if (pq) PQH_HIP(ctx, hipMemcpyAsync(dp.p, pq, (size_t)n * pq_m, hipMemcpyHostToDevice, ctx->stream));
    std::vector<uint32_t> targets((size_t)(n > 0 ? 2 * n : 1));
    std::vector<int> counts((size_t)(n > 0 ? n : 1));
    long long ne = 0;
    if ((rc = pqh_mst_build(ctx, di.p, dd.p, n, num_nn, take, pq ? dp.p : nullptr, pq_m,
                            pq ? penalty : 0.0f, targets.data(), counts.data(), &ne)))
        return rc;
    {   // mst.tree
        FILE* f = fopen(path_of(out_template, "mst.tree").c_str(), "wb");
        if (!f) return PQH_ERR_ARG;
        bool ok = fwrite(&n, sizeof(long long), 1, f) == 1 && fwrite(&ne, sizeof(long long), 1, f) == 1 &&
                  fwrite(targets.data(), sizeof(uint32_t), (size_t)ne, f) == (size_t)ne &&
                  fwrite(counts.data(), sizeof(int), (size_t)n, f) == (size_t)n;
        if (fclose(f) != 0 || !ok) return PQH_ERR_ARG;
    }
    if (!pq) return PQH_OK;   // the estimate needs the PQ codes (mst_builder.c:118)
    // tree_estimate_huffman_encoding (mst.c:496-530): DFS order, parent -> child code pairs
    std::vector<uint32_t> vertices((size_t)n);
    std::vector<int> nch((size_t)n);
    std::vector<long long> parents((size_t)n);
    const int roots = pqh_tree_order(n, ne, targets.data(), counts.data(), vertices.data(),
                                     nch.data(), parents.data());
    if (roots < 0) return roots;
    const int ks = 256;
    std::vector<double> stats((size_t)pq_m * ks * ks, 0.0);
    for (long long p = 0; p < n; ++p) {
        if (parents[p] < 0) continue;
        const byte_t* pr = pq + (size_t)parents[p] * pq_m;
        const byte_t* cu = pq + (size_t)vertices[p] * pq_m;
        for (int i = 0; i < pq_m; ++i) stats[(size_t)i * ks * ks + (size_t)pr[i] * ks + cu[i]] += 1.0;
    }
    huffman_stats_t is, cs;
    huffman_stats_init(&is, n, pq_m, ks);
    is.num_roots = roots;
    for (int i = 0; i < pq_m; ++i) {
        huffman_codebook_t cb;
        huffman_codebook_context_encode_init(&cb, ks, stats.data() + (size_t)i * ks * ks);
        huffman_stats_push(&is, i, huffman_estimate_size(&cb, stats.data() + (size_t)i * ks * ks));
        huffman_codebook_destroy(&cb);
    }
    int alphabet = 0;   // tree_collect_num_children_stats (mst.c:407-440)
    for (long long p = 0; p < n; ++p) alphabet = nch[p] > alphabet ? nch[p] : alphabet;
    ++alphabet;
    printf("Max num children: %d\n", alphabet);
    std::vector<double> cstats((size_t)alphabet, 0.0);
    for (long long p = 0; p < n; ++p) cstats[(size_t)nch[p]] += 1.0;
    huffman_codebook_t cb;
    huffman_codebook_encode_init(&cb, alphabet, cstats.data());
    const double cest = huffman_estimate_size(&cb, cstats.data());
    huffman_codebook_destroy(&cb);
    huffman_stats_init(&cs, n, 1, alphabet);
    huffman_stats_push(&cs, 0, cest);
    huffman_stats_print(&is);
    huffman_stats_print_filename(&is, path_of(out_template, "stats.json").c_str());
    huffman_stats_print_filename(&cs, path_of(out_template, "stats_num_children.json").c_str());
    huffman_stats_destroy(&is);
    huffman_stats_destroy(&cs);
    return PQH_OK;
}
