// pqh_tree.cpp -- host side of tree-ordered context coding.
//
// The DFS order of a stored spanning forest (mst.c:290-364, tree_collect_vertices_dfs) and
// each row's coding context -- the vertex on top of the traverser stack when the row is
// coded (mst.c:366-405, tree_traverser_*; driven by huffman_encoder.c:240-286).  Both are a
// sequential stack walk over the forest's adjacency lists, O(N) host work like the code-book
// heaps; the rows themselves are gathered, counted and coded on the GPU (pqh_huff.hip).
#include <cstdint>
#include <vector>

#include "pqh_internal.h"

int pqh_tree_order(long long num_vertices, long long num_edges, const uint32_t* edge_targets,
                   const int* children_counts, uint32_t* vertices, int* num_children,
                   long long* parents) {
    if (num_vertices < 0 || num_edges < 0 || (num_vertices > 0 && !children_counts) ||
        (num_edges > 0 && !edge_targets) || (num_vertices > 0 && (!vertices || !num_children)))
        return PQH_ERR_ARG;
    if (num_vertices == 0) return 0;
    // adjacency list of vertex i = edge_targets[first[i], first[i] + children_counts[i])
    // (restore_tree_edges_pointers, mst.c:52-61)
    // (a forest has < 2^32 edges: 32-bit offsets halve the walk's random-access footprint)
    if (num_edges >= (1LL << 32) || num_vertices >= (1LL << 32) - 1) return PQH_ERR_ARG;
    std::vector<uint32_t> first((size_t)num_vertices + 1, 0);
    long long total = 0;
    for (long long i = 0; i < num_vertices; ++i) {
        if (children_counts[i] < 0) return PQH_ERR_ARG;
        total += children_counts[i];
        if (total > num_edges) return PQH_ERR_ARG;
        first[i + 1] = (uint32_t)total;
    }
    if (total != num_edges) return PQH_ERR_ARG;
    for (long long e = 0; e < num_edges; ++e)
        if ((long long)edge_targets[e] >= num_vertices) return PQH_ERR_ARG;

    // DFS with marking on push; roots are the lowest unvisited ids (mst.c:303-353).
    // mark[v] = 0 unvisited, else 1 + the DFS position of the vertex that pushed it, so one
    // pass over the adjacency list both pushes and counts: the reference counts unvisited
    // neighbours before pushing any (:322-333), so a target repeated in one list counts once
    // per repeat -- a repeat is a target already marked by this same vertex.
    std::vector<uint32_t> stack((size_t)num_vertices);
    std::vector<uint32_t> mark((size_t)num_vertices, 0);
    long long processed = 0, stack_size = 0, children_sum = 0;
    uint32_t next_root = 0;
    int num_roots = 0;
    while (processed < num_vertices) {
        if (stack_size == 0) {
            while ((long long)next_root < num_vertices && mark[next_root]) ++next_root;
            stack[stack_size++] = next_root;
            mark[next_root] = UINT32_MAX;   // pushed by no vertex
            ++num_roots;
        }
        const uint32_t cur = stack[--stack_size];
        const uint32_t stamp = (uint32_t)processed + 1;
        vertices[processed] = cur;
        int kids = 0;
        for (uint32_t e = first[cur]; e < first[cur + 1]; ++e) {
            const uint32_t t = edge_targets[e];
            const uint32_t mt = mark[t];
            if (!mt) {
                mark[t] = stamp;
                stack[stack_size++] = t;
                ++kids;
            } else if (mt == stamp) {
                ++kids;
            }
        }
        num_children[processed] = kids;
        children_sum += kids;
        ++processed;
    }
    // the reference asserts this (mst.c:357): a duplicated edge breaks the child counts
    if (children_sum != num_vertices - num_roots) return PQH_ERR_ARG;

    // coding context of each stream row: the traverser's active parent (mst.c:383-405)
    if (parents) {
        struct item { uint32_t vertex; int left; };
        std::vector<item> tstack;
        tstack.reserve((size_t)num_vertices);
        for (long long p = 0; p < num_vertices; ++p) {
            parents[p] = tstack.empty() ? -1 : (long long)tstack.back().vertex;
            if (!tstack.empty() && --tstack.back().left == 0) tstack.pop_back();
            if (num_children[p]) tstack.push_back({vertices[p], num_children[p]});
        }
    }
    return num_roots;
}

// Decode-side index of a tree stream: the stream position of each row's context
// (the traverser of huffman_decoder.c:214-247, pushing positions), and per chunk of C rows
// the rows whose context lies before the chunk -- ext_offsets[j] .. ext_offsets[j + 1] index
// ext_positions, the context positions in row order.  Returns the ext count.
long long pqh_tree_ext_index(long long n, const int* num_children, int chunk_vectors,
                             long long* parent_pos, long long* ext_offsets,
                             long long* ext_positions) {
    if (n < 0 || chunk_vectors <= 0 || (n > 0 && (!num_children || !parent_pos || !ext_offsets)))
        return PQH_ERR_ARG;
    struct item { long long pos; int left; };
    std::vector<item> tstack;
    long long ext = 0;
    for (long long p = 0; p < n; ++p) {
        if (p % chunk_vectors == 0) ext_offsets[p / chunk_vectors] = ext;
        const long long pp = tstack.empty() ? -1 : tstack.back().pos;
        parent_pos[p] = pp;
        if (pp >= 0 && pp < p - p % chunk_vectors) {
            if (ext_positions) ext_positions[ext] = pp;
            ++ext;
        }
        if (!tstack.empty() && --tstack.back().left == 0) tstack.pop_back();
        if (num_children[p] < 0) return PQH_ERR_ARG;
        if (num_children[p]) tstack.push_back({p, num_children[p]});
    }
    if (n > 0) ext_offsets[(n + chunk_vectors - 1) / chunk_vectors] = ext;
    return ext;
}
