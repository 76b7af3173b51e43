// pqh_files.cpp -- whole-file encode/decode on top of the pqh GPU calls, used by the CLI
// tools (csrc/tools).  Produces exactly the reference's files (huffman_encoder.c:306-439):
//   huffman_codebooks.bin  u32 m + m x huffman_codebook_save
//   huffman_indices.bin    u64 N + stream (zero padded)
//   huffman_stats.txt      JSON line appended (stats.c)
// plus the decode sidecar huffman_chunks.bin (pqh extension, see pqh.h).
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "pqh_internal.h"
#include "stats.h"

namespace {

struct Sidecar {
    char magic[4];
    uint32_t version, m, k, context, chunk_vectors, raw_first;
    uint64_t n, chunks;
};

// huffman_tree_chunks.bin: the tree decoder's index (pqh extension) -- chunk bit offsets
// and the context rows that precede each chunk (pqh_tree_ext_index order)
struct TreeSidecar {
    char magic[4];
    uint32_t version, m, chunk_vectors;
    uint64_t n, chunks, ext;
};
constexpr int kTreeFileChunk = 16;

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

}  // namespace

extern "C" int pqh_encode_files(const unsigned char* codes, long long n, int m,
                                const pqh_encode_options_t* options, const char* out_prefix) {
    const int k = 256;
    pqh_encode_options_t opt = {1, 1, 64, 0};
    if (options) opt = *options;
    if (!codes || n < 0 || m <= 0 || m > 16 || !out_prefix) return PQH_ERR_ARG;
    if (opt.chunk_vectors <= 0) opt.chunk_vectors = 64;
    if (opt.context && n == 0) return PQH_ERR_ARG;  // the reference asserts (huffman_encoder.c:198)
    CtxGuard g;
    int rc = pqh_ctx_create(&g.ctx, 0);
    if (rc) return rc;
    pqh_ctx* ctx = g.ctx;
    const long long items = opt.context ? (long long)k * k : k;
    DevBuf<unsigned char> d_codes;
    DevBuf<uint32_t> d_counts;
    if ((rc = d_codes.alloc(ctx, (size_t)n * m)) || (rc = d_counts.alloc(ctx, (size_t)m * items)))
        return rc;
    PQH_HIP(ctx, hipMemcpyAsync(d_codes.p, codes, (size_t)n * m, hipMemcpyHostToDevice, ctx->stream));
    if (opt.sort) {
        DevBuf<unsigned char> tmp;
        if ((rc = tmp.alloc(ctx, (size_t)n * m))) return rc;
        if ((rc = pqh_sort_rows(ctx, d_codes.p, n, m, tmp.p))) return rc;
    }
    PQH_HIP(ctx, hipMemsetAsync(d_counts.p, 0, (size_t)m * items * 4, ctx->stream));
    if ((rc = pqh_histogram(ctx, d_codes.p, n, m, k, opt.context, nullptr, d_counts.p))) return rc;
    // codes are built on the GPU from the device histogram (pqh_tables_build); the host
    // copies feed huffman_codebooks.bin and the stats line
    pqh_tables_t* tab = nullptr;
    if ((rc = pqh_tables_alloc(ctx, m, k, opt.context, &tab))) return rc;
    rc = pqh_tables_build(ctx, tab, d_counts.p);
    std::vector<huffman_codebook_t> cbs(m);
    if (!rc) rc = pqh_tables_codebooks(ctx, tab, cbs.data());
    if (rc) {
        pqh_tables_destroy(tab);
        return rc;
    }
    std::vector<uint32_t> hc((size_t)m * items);
    PQH_HIP(ctx, hipMemcpyAsync(hc.data(), d_counts.p, hc.size() * 4, hipMemcpyDeviceToHost, ctx->stream));
    PQH_HIP(ctx, hipStreamSynchronize(ctx->stream));
    std::vector<double> counts(hc.begin(), hc.end());

    huffman_stats_t st;
    huffman_stats_init(&st, n, m, k);
    st.num_roots = opt.context ? 1 : 0;
    for (int i = 0; i < m; ++i)
        huffman_stats_push(&st, i, huffman_estimate_size(&cbs[i], counts.data() + i * items));
    huffman_stats_print(&st);
    huffman_stats_print_filename(&st, path_of(out_prefix, "huffman_stats.txt").c_str());
    huffman_stats_destroy(&st);
    if (opt.only_estimate) {
        for (auto& cb : cbs) huffman_codebook_destroy(&cb);
        pqh_tables_destroy(tab);
        return PQH_OK;
    }

    FILE* cf = fopen(path_of(out_prefix, "huffman_codebooks.bin").c_str(), "wb");
    if (!cf) {
        pqh_tables_destroy(tab);
        return pqh_set_error(ctx, PQH_ERR_ARG, "cannot write codebooks");
    }
    uint32_t mu = (uint32_t)m;
    bool cok = fwrite(&mu, 4, 1, cf) == 1;
    for (int i = 0; i < m; ++i) huffman_codebook_save(&cbs[i], cf);
    cok = !ferror(cf) && cok;
    cok = fclose(cf) == 0 && cok;
    for (auto& cb : cbs) huffman_codebook_destroy(&cb);
    if (!cok) {
        pqh_tables_destroy(tab);
        return pqh_set_error(ctx, PQH_ERR_ARG, "cannot write codebooks");
    }

    DevBuf<unsigned long long> d_total;
    const long long chunks = (n + opt.chunk_vectors - 1) / opt.chunk_vectors;
    DevBuf<unsigned long long> d_coff;
    DevBuf<unsigned char> d_cprev;
    if ((rc = d_total.alloc(ctx, 1)) || (rc = d_coff.alloc(ctx, chunks + 1)) ||
        (rc = d_cprev.alloc(ctx, (size_t)(chunks + 1) * m))) {
        pqh_tables_destroy(tab);
        return rc;
    }
    rc = pqh_encode_size(ctx, tab, d_codes.p, n, 1, nullptr, d_total.p);
    unsigned long long total = 0;
    if (!rc) {
        PQH_HIP(ctx, hipMemcpyAsync(&total, d_total.p, 8, hipMemcpyDeviceToHost, ctx->stream));
        PQH_HIP(ctx, hipStreamSynchronize(ctx->stream));
    }
    const unsigned long long bytes = (total + 7) / 8, wbytes = ((total + 31) / 32) * 4 + 4;
    DevBuf<unsigned char> d_out;
    if (!rc) rc = d_out.alloc(ctx, wbytes);
    if (!rc) {
        PQH_HIP(ctx, hipMemsetAsync(d_out.p, 0, wbytes, ctx->stream));
        rc = pqh_encode_write(ctx, tab, d_codes.p, n, 1, nullptr, 0, d_out.p, wbytes,
                              opt.chunk_vectors, d_coff.p, d_cprev.p, nullptr);
        if (!rc) rc = pqh_encode_status(ctx);
    }
    pqh_tables_destroy(tab);
    if (rc) return rc;
    std::vector<unsigned char> stream(bytes + 1);
    std::vector<unsigned long long> coff(chunks + 1);
    std::vector<unsigned char> cprev((size_t)(chunks + 1) * m);
    PQH_HIP(ctx, hipMemcpyAsync(stream.data(), d_out.p, bytes, hipMemcpyDeviceToHost, ctx->stream));
    PQH_HIP(ctx, hipMemcpyAsync(coff.data(), d_coff.p, chunks * 8, hipMemcpyDeviceToHost, ctx->stream));
    PQH_HIP(ctx, hipMemcpyAsync(cprev.data(), d_cprev.p, (size_t)chunks * m, hipMemcpyDeviceToHost,
                                ctx->stream));
    PQH_HIP(ctx, hipStreamSynchronize(ctx->stream));

    FILE* ef = fopen(path_of(out_prefix, "huffman_indices.bin").c_str(), "wb");
    if (!ef) return pqh_set_error(ctx, PQH_ERR_ARG, "cannot write indices");
    unsigned long long nn = (unsigned long long)n;
    bool wok = fwrite(&nn, 8, 1, ef) == 1;
    wok = fwrite(stream.data(), 1, bytes, ef) == bytes && wok;
    wok = fclose(ef) == 0 && wok;
    if (!wok) return pqh_set_error(ctx, PQH_ERR_ARG, "cannot write indices");

    // the sidecar is optional (the decoder rebuilds the chunk index without it), but a
    // partly written one is an error
    FILE* sf = fopen(path_of(out_prefix, "huffman_chunks.bin").c_str(), "wb");
    if (sf) {
        Sidecar h;
        memcpy(h.magic, "PQHC", 4);
        h.version = 1;
        h.m = m;
        h.k = k;
        h.context = opt.context;
        h.chunk_vectors = opt.chunk_vectors;
        h.raw_first = 1;
        h.n = n;
        h.chunks = chunks;
        bool sok = fwrite(&h, sizeof(h), 1, sf) == 1;
        sok = (long long)fwrite(coff.data(), 8, chunks, sf) == chunks && sok;
        if (opt.context) sok = fwrite(cprev.data(), 1, (size_t)chunks * m, sf) == (size_t)chunks * m && sok;
        sok = fclose(sf) == 0 && sok;
        if (!sok) return pqh_set_error(ctx, PQH_ERR_ARG, "cannot write huffman_chunks.bin");
    }
    return PQH_OK;
}

extern "C" int pqh_decode_files(const char* in_prefix, unsigned char** codes_out, long long* n_out,
                                int* m_out) {
    if (!in_prefix || !codes_out || !n_out || !m_out) return PQH_ERR_ARG;
    *codes_out = nullptr;
    FILE* cf = fopen(path_of(in_prefix, "huffman_codebooks.bin").c_str(), "rb");
    if (!cf) return PQH_ERR_ARG;
    uint32_t m = 0;
    if (fread(&m, 4, 1, cf) != 1 || m == 0 || m > 16) {
        fclose(cf);
        return PQH_ERR_CORRUPT;
    }
    std::vector<huffman_codebook_t> cbs(m);
    for (uint32_t i = 0; i < m; ++i) huffman_codebook_load(&cbs[i], cf);
    fclose(cf);
    FILE* ef = fopen(path_of(in_prefix, "huffman_indices.bin").c_str(), "rb");
    if (!ef) return PQH_ERR_ARG;
    unsigned long long n = 0;
    if (fread(&n, 8, 1, ef) != 1) n = 0;
    fseek(ef, 0, SEEK_END);
    const long long fsize = ftell(ef);
    fseek(ef, 8, SEEK_SET);
    const unsigned long long bytes = fsize > 8 ? (unsigned long long)(fsize - 8) : 0;
    const unsigned long long wbytes = ((bytes + 3) / 4) * 4 + 8;
    std::vector<unsigned char> stream(wbytes, 0);
    if (bytes && fread(stream.data(), 1, bytes, ef) != bytes) {
        fclose(ef);
        return PQH_ERR_CORRUPT;
    }
    fclose(ef);

    CtxGuard g;
    int rc = pqh_ctx_create(&g.ctx, 0);
    if (rc) return rc;
    pqh_ctx* ctx = g.ctx;
    pqh_tables_t* tab = nullptr;
    rc = pqh_tables_create(ctx, cbs.data(), (int)m, &tab);
    const int context = cbs[0].is_context;
    const int k = cbs[0].alphabet_size;
    for (auto& cb : cbs) huffman_codebook_destroy(&cb);
    if (rc) return rc;
    const size_t esz = k <= 256 ? 1 : 2;

    // chunk index: sidecar when it matches, else a host walk of the stream
    int C = 64;
    std::vector<unsigned long long> coff;
    std::vector<unsigned char> cprev;
    bool have = false;
    FILE* sf = fopen(path_of(in_prefix, "huffman_chunks.bin").c_str(), "rb");
    if (sf) {
        Sidecar h;
        if (fread(&h, sizeof(h), 1, sf) == 1 && !memcmp(h.magic, "PQHC", 4) && h.n == n &&
            h.m == m && h.context == (uint32_t)context && h.chunk_vectors > 0 && h.raw_first == 1) {
            C = (int)h.chunk_vectors;
            coff.resize(h.chunks + 1);
            cprev.resize((h.chunks + 1) * m * esz);
            have = fread(coff.data(), 8, h.chunks, sf) == h.chunks;
            if (have && context) have = fread(cprev.data(), esz, h.chunks * m, sf) == h.chunks * m;
        }
        fclose(sf);
    }
    const long long chunks = ((long long)n + C - 1) / C;
    if (!have) {
        coff.assign(chunks + 1, 0);
        cprev.assign((chunks + 1) * m * esz, 0);
        rc = pqh_chunk_index_host(tab, stream.data(), bytes, (long long)n, 1, C, coff.data(),
                                  cprev.data());
        if (rc) {
            pqh_tables_destroy(tab);
            return rc;
        }
    }
    DevBuf<unsigned char> d_stream, d_cprev, d_codes;
    DevBuf<unsigned long long> d_coff;
    if ((rc = d_stream.alloc(ctx, wbytes)) || (rc = d_coff.alloc(ctx, chunks + 1)) ||
        (rc = d_cprev.alloc(ctx, (chunks + 1) * m * esz)) || (rc = d_codes.alloc(ctx, n * m * esz))) {
        pqh_tables_destroy(tab);
        return rc;
    }
    PQH_HIP(ctx, hipMemcpyAsync(d_stream.p, stream.data(), wbytes, hipMemcpyHostToDevice, ctx->stream));
    PQH_HIP(ctx, hipMemcpyAsync(d_coff.p, coff.data(), (chunks + 1) * 8, hipMemcpyHostToDevice, ctx->stream));
    PQH_HIP(ctx, hipMemcpyAsync(d_cprev.p, cprev.data(), (chunks + 1) * m * esz, hipMemcpyHostToDevice,
                                ctx->stream));
    rc = pqh_decode(ctx, tab, d_stream.p, wbytes, (long long)n, 1, C, d_coff.p, d_cprev.p, d_codes.p);
    if (!rc) rc = pqh_decode_status(ctx);
    pqh_tables_destroy(tab);
    if (rc) return rc;
    unsigned char* out = (unsigned char*)malloc(n * m * esz + 1);
    PQH_HIP(ctx, hipMemcpy(out, d_codes.p, n * m * esz, hipMemcpyDeviceToHost));
    *codes_out = out;
    *n_out = (long long)n;
    *m_out = (int)m;
    return PQH_OK;
}

// huffman_encoder --tree <mst.tree> (huffman_encoder.c:321-375, :398-428): tree order and
// contexts on the device (pqh_tree_order_device; the host walk for a non-forest), rows gathered, counted and coded on the GPU, the
// children stream coded by the GPU encoder with the host-built children code book.
// Writes huffman_codebooks.bin, huffman_indices.bin, huffman_stats.txt (appended),
// huffman_children_codebooks.bin, huffman_children.bin, huffman_children_stats.txt.
extern "C" int pqh_encode_tree_files(const unsigned char* codes, long long n, int m, int sort,
                                     const char* tree_path, const char* out_prefix) {
    const int k = 256;
    if (!codes || n <= 0 || m <= 0 || m > 16 || !tree_path || !out_prefix) return PQH_ERR_ARG;
    // tree_load_file (mst.c:273-288): i64 N, i64 E, u32 targets[E], i32 counts[N]
    FILE* tf = fopen(tree_path, "rb");
    if (!tf) return PQH_ERR_ARG;
    long long nv = 0, ne = 0;
    bool ok = fread(&nv, 8, 1, tf) == 1 && fread(&ne, 8, 1, tf) == 1 && nv == n && ne >= 0;
    std::vector<uint32_t> targets(ok ? (size_t)ne : 0);
    std::vector<int> adj(ok ? (size_t)nv : 0);
    ok = ok && fread(targets.data(), 4, (size_t)ne, tf) == (size_t)ne &&
         fread(adj.data(), 4, (size_t)nv, tf) == (size_t)nv;
    fclose(tf);
    if (!ok) return PQH_ERR_ARG;
    std::vector<int> nch(n);

    CtxGuard g;
    int rc = pqh_ctx_create(&g.ctx, 0);
    if (rc) return rc;
    pqh_ctx* ctx = g.ctx;
    const long long items = (long long)k * k;
    DevBuf<unsigned char> d_codes, d_rows;
    DevBuf<uint16_t> d_prev;
    DevBuf<uint32_t> d_vert, d_counts, d_targets;
    DevBuf<long long> d_par;
    DevBuf<int> d_adj, d_nch;
    if ((rc = d_codes.alloc(ctx, (size_t)n * m)) || (rc = d_rows.alloc(ctx, (size_t)n * m)) ||
        (rc = d_prev.alloc(ctx, (size_t)n * m)) || (rc = d_vert.alloc(ctx, n)) ||
        (rc = d_par.alloc(ctx, n)) || (rc = d_counts.alloc(ctx, (size_t)m * items)))
        return rc;
    PQH_HIP(ctx, hipMemcpyAsync(d_codes.p, codes, (size_t)n * m, hipMemcpyHostToDevice, ctx->stream));
    // tree order (tree_collect_vertices_dfs + the traverser's parents) on the device; a file
    // that is not a forest (a cycle, a repeated edge) takes the host walk, which reproduces
    // the reference's DFS on any graph.  PQH_TREE_ORDER=host forces the host walk.
    int roots = -1;
    const char* tmode = getenv("PQH_TREE_ORDER");
    if (!(tmode && !strcmp(tmode, "host"))) {
        if ((rc = d_targets.alloc(ctx, ne > 0 ? ne : 1)) || (rc = d_adj.alloc(ctx, n)) ||
            (rc = d_nch.alloc(ctx, n)))
            return rc;
        if (ne > 0)
            PQH_HIP(ctx, hipMemcpyAsync(d_targets.p, targets.data(), (size_t)ne * 4,
                                        hipMemcpyHostToDevice, ctx->stream));
        PQH_HIP(ctx, hipMemcpyAsync(d_adj.p, adj.data(), (size_t)n * 4, hipMemcpyHostToDevice, ctx->stream));
        int r = 0;
        rc = pqh_tree_order_device(ctx, n, ne, d_targets.p, d_adj.p, d_vert.p, d_nch.p, d_par.p, &r);
        if (rc == PQH_OK) {
            roots = r;
            PQH_HIP(ctx, hipMemcpyAsync(nch.data(), d_nch.p, (size_t)n * 4, hipMemcpyDeviceToHost,
                                        ctx->stream));
        } else if (rc != PQH_ERR_UNSUPPORTED) {
            return rc;
        }
    }
    if (roots < 0) {
        std::vector<uint32_t> vert(n);
        std::vector<long long> par(n);
        roots = pqh_tree_order(n, ne, targets.data(), adj.data(), vert.data(), nch.data(), par.data());
        if (roots < 0) return roots;
        PQH_HIP(ctx, hipMemcpyAsync(d_vert.p, vert.data(), (size_t)n * 4, hipMemcpyHostToDevice, ctx->stream));
        PQH_HIP(ctx, hipMemcpyAsync(d_par.p, par.data(), (size_t)n * 8, hipMemcpyHostToDevice, ctx->stream));
        PQH_HIP(ctx, hipStreamSynchronize(ctx->stream));
    }
    if (sort) {   // the CLI sorts before applying the tree (huffman_encoder.c:313-325)
        DevBuf<unsigned char> tmp;
        if ((rc = tmp.alloc(ctx, (size_t)n * m))) return rc;
        if ((rc = pqh_sort_rows(ctx, d_codes.p, n, m, tmp.p))) return rc;
    }
    if ((rc = pqh_tree_gather(ctx, d_codes.p, n, m, k, d_vert.p, d_par.p, d_rows.p, d_prev.p)) ||
        (rc = pqh_tree_status(ctx)))
        return rc;
    PQH_HIP(ctx, hipMemsetAsync(d_counts.p, 0, (size_t)m * items * 4, ctx->stream));
    if ((rc = pqh_histogram_tree(ctx, d_rows.p, d_prev.p, n, m, k, d_counts.p))) return rc;
    pqh_tables_t* tab = nullptr;
    if ((rc = pqh_tables_alloc(ctx, m, k, 1, &tab))) return rc;
    rc = pqh_tables_build(ctx, tab, d_counts.p);
    std::vector<huffman_codebook_t> cbs(m);
    if (!rc) rc = pqh_tables_codebooks(ctx, tab, cbs.data());
    if (rc) {
        pqh_tables_destroy(tab);
        return rc;
    }
    std::vector<uint32_t> hc((size_t)m * items);
    PQH_HIP(ctx, hipMemcpyAsync(hc.data(), d_counts.p, hc.size() * 4, hipMemcpyDeviceToHost, ctx->stream));
    PQH_HIP(ctx, hipStreamSynchronize(ctx->stream));
    std::vector<double> counts(hc.begin(), hc.end());

    // children code book + stream (huffman_encoder.c:343-375)
    int alphabet = 0;
    for (long long p = 0; p < n; ++p) alphabet = nch[p] > alphabet ? nch[p] : alphabet;
    ++alphabet;
    printf("Max num children: %d\n", alphabet);
    if (alphabet > 4096) {
        for (auto& cb : cbs) huffman_codebook_destroy(&cb);
        pqh_tables_destroy(tab);
        return pqh_set_error(ctx, PQH_ERR_UNSUPPORTED, "more than 4095 children at one vertex");
    }
    std::vector<double> ccounts(alphabet, 0.0);
    for (long long p = 0; p < n; ++p) ccounts[nch[p]] += 1.0;
    huffman_codebook_t ccb;
    huffman_codebook_encode_init(&ccb, alphabet, ccounts.data());
    {
        FILE* f = fopen(path_of(out_prefix, "huffman_children_codebooks.bin").c_str(), "wb");
        bool ok = f != nullptr;
        if (f) {
            huffman_codebook_save(&ccb, f);
            ok = !ferror(f);
            ok = fclose(f) == 0 && ok;
        }
        if (!ok) {
            for (auto& cb : cbs) huffman_codebook_destroy(&cb);
            huffman_codebook_destroy(&ccb);
            pqh_tables_destroy(tab);
            return pqh_set_error(ctx, PQH_ERR_ARG, "cannot write huffman_children_codebooks.bin");
        }
        huffman_stats_t cst;
        huffman_stats_init(&cst, n, 1, k);
        huffman_stats_push(&cst, 0, huffman_estimate_size(&ccb, ccounts.data()));
        huffman_stats_print_filename(&cst, path_of(out_prefix, "huffman_children_stats.txt").c_str());
        huffman_stats_destroy(&cst);
    }

    huffman_stats_t st;
    huffman_stats_init(&st, n, m, k);
    st.num_roots = roots;
    double total_bits = 8.0 * m * roots;
    for (int i = 0; i < m; ++i) {
        const double e = huffman_estimate_size(&cbs[i], counts.data() + i * items);
        huffman_stats_push(&st, i, e);
        total_bits += e;
    }
    huffman_stats_print(&st);
    huffman_stats_print_filename(&st, path_of(out_prefix, "huffman_stats.txt").c_str());
    huffman_stats_destroy(&st);
    FILE* cf = fopen(path_of(out_prefix, "huffman_codebooks.bin").c_str(), "wb");
    bool cf_ok = cf != nullptr;
    if (cf) {
        uint32_t mu = (uint32_t)m;
        cf_ok = fwrite(&mu, 4, 1, cf) == 1;
        for (int i = 0; i < m; ++i) huffman_codebook_save(&cbs[i], cf);
        cf_ok = !ferror(cf) && cf_ok;
        cf_ok = fclose(cf) == 0 && cf_ok;
    }
    for (auto& cb : cbs) huffman_codebook_destroy(&cb);
    if (!cf_ok) {
        huffman_codebook_destroy(&ccb);
        pqh_tables_destroy(tab);
        return pqh_set_error(ctx, PQH_ERR_ARG, "cannot write huffman_codebooks.bin");
    }

    // the row stream (encode_tree_data, huffman_encoder.c:240-286)
    const unsigned long long cap = ((unsigned long long)total_bits + 31) / 32 * 4 + 64;
    DevBuf<unsigned char> d_out;
    DevBuf<unsigned long long> d_total, d_coff;
    unsigned long long bits = 0;
    const long long chunks = (n + kTreeFileChunk - 1) / kTreeFileChunk;
    if ((rc = d_coff.alloc(ctx, chunks + 1))) {
        pqh_tables_destroy(tab);
        huffman_codebook_destroy(&ccb);
        return rc;
    }
    if (!(rc = d_out.alloc(ctx, cap)) && !(rc = d_total.alloc(ctx, 1)))
        rc = pqh_encode_tree_write(ctx, tab, d_rows.p, d_prev.p, n, 0, d_out.p, cap,
                                   kTreeFileChunk, d_coff.p, d_total.p);
    if (!rc) rc = pqh_encode_status(ctx);
    pqh_tables_destroy(tab);
    std::vector<unsigned char> stream;
    if (!rc) {
        PQH_HIP(ctx, hipMemcpyAsync(&bits, d_total.p, 8, hipMemcpyDeviceToHost, ctx->stream));
        PQH_HIP(ctx, hipStreamSynchronize(ctx->stream));
        stream.resize((bits + 7) / 8 + 1);
        PQH_HIP(ctx, hipMemcpyAsync(stream.data(), d_out.p, (bits + 7) / 8, hipMemcpyDeviceToHost,
                                    ctx->stream));
    }
    // the children stream: one non-context part, u8 or u16 symbols
    pqh_tables_t* ctab = nullptr;
    const size_t esz = alphabet <= 256 ? 1 : 2;
    DevBuf<unsigned char> d_cc, d_cout;
    std::vector<unsigned char> cstream;
    unsigned long long cbits = 0;
    if (!rc) rc = pqh_tables_create(ctx, &ccb, 1, &ctab);
    if (!rc) {
        std::vector<unsigned char> cc((size_t)n * esz);
        for (long long p = 0; p < n; ++p) {
            if (esz == 1) cc[p] = (unsigned char)nch[p];
            else reinterpret_cast<uint16_t*>(cc.data())[p] = (uint16_t)nch[p];
        }
        double cb_bits = huffman_estimate_size(&ccb, ccounts.data());
        const unsigned long long ccap = ((unsigned long long)cb_bits + 31) / 32 * 4 + 64;
        if (!(rc = d_cc.alloc(ctx, cc.size())) && !(rc = d_cout.alloc(ctx, ccap))) {
            PQH_HIP(ctx, hipMemcpyAsync(d_cc.p, cc.data(), cc.size(), hipMemcpyHostToDevice, ctx->stream));
            rc = pqh_encode_write(ctx, ctab, d_cc.p, n, 1, nullptr, 0, d_cout.p, ccap, 0, nullptr,
                                  nullptr, d_total.p);
        }
        if (!rc) rc = pqh_encode_status(ctx);
        if (!rc) {
            PQH_HIP(ctx, hipMemcpyAsync(&cbits, d_total.p, 8, hipMemcpyDeviceToHost, ctx->stream));
            PQH_HIP(ctx, hipStreamSynchronize(ctx->stream));
            cstream.resize((cbits + 7) / 8 + 1);
            PQH_HIP(ctx, hipMemcpyAsync(cstream.data(), d_cout.p, (cbits + 7) / 8,
                                        hipMemcpyDeviceToHost, ctx->stream));
            PQH_HIP(ctx, hipStreamSynchronize(ctx->stream));
        }
    }
    if (ctab) pqh_tables_destroy(ctab);
    huffman_codebook_destroy(&ccb);
    if (rc) return rc;
    // decode sidecar: chunk offsets + the context rows that precede each chunk
    std::vector<unsigned long long> coff(chunks);
    std::vector<unsigned char> rows((size_t)n * m);
    PQH_HIP(ctx, hipMemcpyAsync(coff.data(), d_coff.p, chunks * 8, hipMemcpyDeviceToHost, ctx->stream));
    PQH_HIP(ctx, hipMemcpyAsync(rows.data(), d_rows.p, rows.size(), hipMemcpyDeviceToHost, ctx->stream));
    PQH_HIP(ctx, hipStreamSynchronize(ctx->stream));
    std::vector<long long> pp(n), eo(chunks + 1);
    const long long ext = pqh_tree_ext_index(n, nch.data(), kTreeFileChunk, pp.data(), eo.data(),
                                             nullptr);
    if (ext < 0) return (int)ext;
    std::vector<long long> ep(ext + 1);
    pqh_tree_ext_index(n, nch.data(), kTreeFileChunk, pp.data(), eo.data(), ep.data());
    FILE* tsf = fopen(path_of(out_prefix, "huffman_tree_chunks.bin").c_str(), "wb");
    if (!tsf) return pqh_set_error(ctx, PQH_ERR_ARG, "cannot write huffman_tree_chunks.bin");
    {
        TreeSidecar h;
        memcpy(h.magic, "PQHT", 4);
        h.version = 1;
        h.m = m;
        h.chunk_vectors = kTreeFileChunk;
        h.n = n;
        h.chunks = chunks;
        h.ext = ext;
        bool ok = fwrite(&h, sizeof(h), 1, tsf) == 1;
        ok = (long long)fwrite(coff.data(), 8, chunks, tsf) == chunks && ok;
        for (long long e = 0; e < ext && ok; ++e)
            ok = fwrite(rows.data() + ep[e] * m, 1, m, tsf) == (size_t)m;
        ok = fclose(tsf) == 0 && ok;
        if (!ok) return pqh_set_error(ctx, PQH_ERR_ARG, "cannot write huffman_tree_chunks.bin");
    }
    FILE* ef = fopen(path_of(out_prefix, "huffman_indices.bin").c_str(), "wb");
    if (!ef) return pqh_set_error(ctx, PQH_ERR_ARG, "cannot write indices");
    unsigned long long nn = (unsigned long long)n;
    bool wok = fwrite(&nn, 8, 1, ef) == 1;
    wok = fwrite(stream.data(), 1, (bits + 7) / 8, ef) == (bits + 7) / 8 && wok;
    wok = fclose(ef) == 0 && wok;
    if (!wok) return pqh_set_error(ctx, PQH_ERR_ARG, "cannot write indices");
    FILE* chf = fopen(path_of(out_prefix, "huffman_children.bin").c_str(), "wb");
    if (!chf) return pqh_set_error(ctx, PQH_ERR_ARG, "cannot write children stream");
    wok = fwrite(cstream.data(), 1, (cbits + 7) / 8, chf) == (cbits + 7) / 8;
    wok = fclose(chf) == 0 && wok;
    if (!wok) return pqh_set_error(ctx, PQH_ERR_ARG, "cannot write children stream");
    return PQH_OK;
}

// huffman_decoder --tree (huffman_decoder.c:174-247) on the GPU: the children stream first
// (GPU decode; its chunk index from a host walk of the table), the traverser index on the
// host, then dec_tree with the encoder's sidecar huffman_tree_chunks.bin (required: a tree
// stream cannot be split into independent chunks without it).  Rows in stream order.
extern "C" int pqh_decode_tree_files(const char* in_prefix, unsigned char** codes_out,
                                     long long* n_out, int* m_out) {
    if (!in_prefix || !codes_out || !n_out || !m_out) return PQH_ERR_ARG;
    *codes_out = nullptr;
    auto slurp = [&](const char* name, long long skip, std::vector<unsigned char>& buf,
                     unsigned long long& bytes) {
        FILE* f = fopen(path_of(in_prefix, name).c_str(), "rb");
        if (!f) return false;
        fseek(f, 0, SEEK_END);
        const long long size = ftell(f);
        fseek(f, skip, SEEK_SET);
        bytes = size > skip ? (unsigned long long)(size - skip) : 0;
        buf.assign(((bytes + 3) / 4) * 4 + 8, 0);
        const bool ok = !bytes || fread(buf.data(), 1, bytes, f) == bytes;
        fclose(f);
        return ok;
    };
    FILE* cf = fopen(path_of(in_prefix, "huffman_codebooks.bin").c_str(), "rb");
    if (!cf) return PQH_ERR_ARG;
    uint32_t m = 0;
    if (fread(&m, 4, 1, cf) != 1 || m == 0 || m > 16) {
        fclose(cf);
        return PQH_ERR_CORRUPT;
    }
    std::vector<huffman_codebook_t> cbs(m);
    for (uint32_t i = 0; i < m; ++i) huffman_codebook_load(&cbs[i], cf);
    fclose(cf);
    huffman_codebook_t ccb;
    FILE* ccf = fopen(path_of(in_prefix, "huffman_children_codebooks.bin").c_str(), "rb");
    if (!ccf) {
        for (auto& cb : cbs) huffman_codebook_destroy(&cb);
        return PQH_ERR_ARG;
    }
    huffman_codebook_load(&ccb, ccf);
    fclose(ccf);
    unsigned long long n = 0;
    {
        FILE* ef = fopen(path_of(in_prefix, "huffman_indices.bin").c_str(), "rb");
        if (!ef || fread(&n, 8, 1, ef) != 1) n = 0;
        if (ef) fclose(ef);
    }
    std::vector<unsigned char> stream, cstream, side;
    unsigned long long bytes = 0, cbytes = 0, sbytes = 0;
    bool ok = n > 0 && slurp("huffman_indices.bin", 8, stream, bytes) &&
              slurp("huffman_children.bin", 0, cstream, cbytes) &&
              slurp("huffman_tree_chunks.bin", 0, side, sbytes) && sbytes >= sizeof(TreeSidecar);
    TreeSidecar h{};
    if (ok) {
        memcpy(&h, side.data(), sizeof(h));
        ok = !memcmp(h.magic, "PQHT", 4) && h.n == n && h.m == m && h.chunk_vectors > 0 &&
             h.chunks == (n + h.chunk_vectors - 1) / h.chunk_vectors &&
             sbytes >= sizeof(h) + h.chunks * 8 + h.ext * m;
    }
    CtxGuard g;
    int rc = ok ? pqh_ctx_create(&g.ctx, 0) : PQH_ERR_ARG;
    pqh_tables_t *tab = nullptr, *ctab = nullptr;
    if (!rc) rc = pqh_tables_create(g.ctx, cbs.data(), (int)m, &tab);
    if (!rc) rc = pqh_tables_create(g.ctx, &ccb, 1, &ctab);
    const int calpha = ccb.alphabet_size;
    for (auto& cb : cbs) huffman_codebook_destroy(&cb);
    huffman_codebook_destroy(&ccb);
    auto fail = [&](int r) {
        if (tab) pqh_tables_destroy(tab);
        if (ctab) pqh_tables_destroy(ctab);
        return r;
    };
    if (rc) return fail(rc);
    pqh_ctx* ctx = g.ctx;
    // children stream -> child counts
    const int CC = 64;
    const long long cchunks = ((long long)n + CC - 1) / CC;
    const size_t cesz = calpha <= 256 ? 1 : 2;
    std::vector<unsigned long long> ccoff(cchunks + 1);
    std::vector<unsigned char> ccprev((cchunks + 1) * cesz);
    if ((rc = pqh_chunk_index_host(ctab, cstream.data(), cbytes, (long long)n, 1, CC, ccoff.data(),
                                   ccprev.data())))
        return fail(rc);
    DevBuf<unsigned char> d_cstream, d_cc, d_stream, d_ext, d_rows;
    DevBuf<unsigned long long> d_ccoff, d_coff;
    DevBuf<long long> d_pp, d_eo;
    if ((rc = d_cstream.alloc(ctx, cstream.size())) || (rc = d_ccoff.alloc(ctx, cchunks + 1)) ||
        (rc = d_cc.alloc(ctx, n * cesz)))
        return fail(rc);
    PQH_HIP(ctx, hipMemcpyAsync(d_cstream.p, cstream.data(), cstream.size(), hipMemcpyHostToDevice, ctx->stream));
    PQH_HIP(ctx, hipMemcpyAsync(d_ccoff.p, ccoff.data(), (cchunks + 1) * 8, hipMemcpyHostToDevice, ctx->stream));
    rc = pqh_decode(ctx, ctab, d_cstream.p, cstream.size(), (long long)n, 1, CC, d_ccoff.p, nullptr,
                    d_cc.p);
    if (!rc) rc = pqh_decode_status(ctx);
    if (rc) return fail(rc);
    // the traverser's index on the device from the decoded child counts; its ext count must
    // agree with the sidecar's
    const int C = (int)h.chunk_vectors;
    if ((rc = d_pp.alloc(ctx, n)) || (rc = d_eo.alloc(ctx, h.chunks + 1))) return fail(rc);
    const long long ext = pqh_tree_ext_index_device(ctx, (long long)n, d_cc.p, (int)cesz, C,
                                                    d_pp.p, d_eo.p, nullptr);
    if (ext < 0 || (unsigned long long)ext != h.ext) return fail(PQH_ERR_CORRUPT);
    if ((rc = d_stream.alloc(ctx, stream.size())) || (rc = d_coff.alloc(ctx, h.chunks + 1)) ||
        (rc = d_ext.alloc(ctx, h.ext * m + 1)) || (rc = d_rows.alloc(ctx, n * m)))
        return fail(rc);
    const unsigned char* sp = side.data() + sizeof(h);
    PQH_HIP(ctx, hipMemcpyAsync(d_stream.p, stream.data(), stream.size(), hipMemcpyHostToDevice, ctx->stream));
    PQH_HIP(ctx, hipMemcpyAsync(d_coff.p, sp, h.chunks * 8, hipMemcpyHostToDevice, ctx->stream));
    if (h.ext)
        PQH_HIP(ctx, hipMemcpyAsync(d_ext.p, sp + h.chunks * 8, h.ext * m, hipMemcpyHostToDevice, ctx->stream));
    rc = pqh_decode_tree(ctx, tab, d_stream.p, bytes, (long long)n, C, d_coff.p, d_pp.p,
                         d_eo.p, d_ext.p, d_rows.p);
    if (!rc) rc = pqh_decode_status(ctx);
    if (rc) return fail(rc);
    fail(0);
    unsigned char* out = (unsigned char*)malloc(n * m + 1);
    PQH_HIP(ctx, hipMemcpy(out, d_rows.p, n * m, hipMemcpyDeviceToHost));
    *codes_out = out;
    *n_out = (long long)n;
    *m_out = (int)m;
    return PQH_OK;
}
