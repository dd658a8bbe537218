// h5_keras.cpp -- minimal, self-contained HDF5 reader for Keras Dense weight files.
//
// Replaces the HighFive-based loader of NeuralNetwork::load
// (reference src/neuralNetwork.cpp:85-151; HighFive >= 2.1, un-vendored,
// src/CMakeLists.txt:8).  Supports exactly what the bundled neuralGeometries/*.h5
// use (h5dump -B -p: superblock v0, v1 object headers, symbol-table groups with v1
// B-trees + local heaps, contiguous or compact IEEE float datasets, no filters) and
// fails with NR_E_FORMAT on anything else.  Group members are visited in HDF5 name
// order, the order HighFive's File::listObjectNames returns and the reference
// iterates (so "dense_10" sorts before "dense_2", exactly as in the reference).
#include "nr_internal.h"

#include <algorithm>
#include <cstdio>
#include <cstring>
#include <map>
#include <new>
#include <string>
#include <vector>

namespace nr {
namespace {

struct H5Error { int code; std::string msg; };

[[noreturn]] void fail(int code, const std::string &m) { throw H5Error{code, m}; }

struct File {
    std::vector<uint8_t> d;
    uint64_t base = 0, sb = 0;
    int so = 8, sl = 8;  // size of offsets / lengths

    void need(uint64_t off, uint64_t n) const {
        if (off > d.size() || n > d.size() - off) fail(NR_E_FORMAT, "HDF5: read past end of file");
    }
    uint64_t uint(uint64_t off, int n) const {
        need(off, n);
        uint64_t v = 0;
        for (int i = n - 1; i >= 0; --i) v = (v << 8) | d[off + i];
        return v;
    }
    uint8_t byte(uint64_t off) const { return (uint8_t)uint(off, 1); }
    uint64_t addr(uint64_t off) const { return uint(off, so); }
    bool undef(uint64_t a) const { return so == 8 ? a == ~0ull : a == ((1ull << (8 * so)) - 1); }
    uint64_t abs(uint64_t a) const { return base + a; }
    std::string cstr(uint64_t off) const {
        need(off, 1);
        const char *p = reinterpret_cast<const char *>(&d[off]);
        size_t n = strnlen(p, d.size() - off);
        return std::string(p, n);
    }
};

struct Msg { uint16_t type; uint64_t off; uint32_t size; uint8_t flags; };

std::vector<Msg> object_messages(const File &f, uint64_t oh_addr) {
    uint64_t p = f.abs(oh_addr);
    f.need(p, 16);
    if (f.d[p] != 1) {
        if (f.d[p] == 'O') fail(NR_E_FORMAT, "HDF5: version-2 object headers (OHDR) unsupported");
        fail(NR_E_FORMAT, "HDF5: unknown object header version");
    }
    uint32_t nmsgs = (uint32_t)f.uint(p + 2, 2);
    uint64_t hsize = f.uint(p + 8, 4);
    std::vector<std::pair<uint64_t, uint64_t>> blocks{{p + 16, hsize}};
    std::vector<Msg> out;
    for (size_t bi = 0; bi < blocks.size() && out.size() < nmsgs; ++bi) {
        uint64_t q = blocks[bi].first, end = q + blocks[bi].second;
        f.need(q, blocks[bi].second);
        while (q + 8 <= end && out.size() < nmsgs) {
            Msg m;
            m.type = (uint16_t)f.uint(q, 2);
            m.size = (uint32_t)f.uint(q + 2, 2);
            m.flags = f.byte(q + 4);
            m.off = q + 8;
            f.need(m.off, m.size);
            if (m.type == 0x10) {  // continuation
                blocks.push_back({f.abs(f.addr(m.off)), f.uint(m.off + f.so, f.sl)});
            }
            out.push_back(m);
            q = m.off + m.size;
        }
    }
    return out;
}

const Msg *find(const std::vector<Msg> &ms, uint16_t type) {
    for (auto &m : ms) if (m.type == type) return &m;
    return nullptr;
}

struct Entry { std::string name; uint64_t oh; };

void walk_btree(const File &f, uint64_t node, uint64_t heap_data, std::vector<Entry> &out, int depth, int &budget) {
    if (depth > 32) fail(NR_E_FORMAT, "HDF5: B-tree too deep");
    if (--budget < 0) fail(NR_E_FORMAT, "HDF5: B-tree has too many nodes (a cycle?)");
    uint64_t p = f.abs(node);
    f.need(p, 8);
    if (memcmp(&f.d[p], "TREE", 4) != 0) fail(NR_E_FORMAT, "HDF5: bad B-tree signature");
    if (f.d[p + 4] != 0) fail(NR_E_FORMAT, "HDF5: B-tree is not a group node");
    int level = f.d[p + 5];
    int used = (int)f.uint(p + 6, 2);
    uint64_t q = p + 8 + 2 * f.so;  // skip siblings
    q += f.sl;                       // key 0
    for (int i = 0; i < used; ++i) {
        uint64_t child = f.addr(q);
        q += f.so + f.sl;            // child, key i+1
        if (level > 0) { walk_btree(f, child, heap_data, out, depth + 1, budget); continue; }
        uint64_t s = f.abs(child);
        f.need(s, 8);
        if (memcmp(&f.d[s], "SNOD", 4) != 0) fail(NR_E_FORMAT, "HDF5: bad symbol-node signature");
        int nsym = (int)f.uint(s + 6, 2);
        uint64_t e = s + 8;
        int esz = 2 * f.so + 4 + 4 + 16;
        for (int k = 0; k < nsym; ++k, e += esz) {
            Entry en;
            en.name = f.cstr(f.abs(heap_data + f.uint(e, f.sl)));
            en.oh = f.addr(e + f.so);
            out.push_back(en);
        }
    }
}

// Members of a group in HDF5 name order; returns false if the object is not a group.
bool group_members(const File &f, uint64_t oh, std::vector<Entry> &out) {
    auto ms = object_messages(f, oh);
    const Msg *st = find(ms, 0x11);
    if (!st) {
        if (find(ms, 0x02) || find(ms, 0x06))
            fail(NR_E_FORMAT, "HDF5: new-style (link-message) groups unsupported");
        return false;
    }
    uint64_t btree = f.addr(st->off), heap = f.addr(st->off + f.so);
    uint64_t h = f.abs(heap);
    f.need(h, 8 + 2 * f.sl + f.so);
    if (memcmp(&f.d[h], "HEAP", 4) != 0) fail(NR_E_FORMAT, "HDF5: bad local heap signature");
    uint64_t heap_data = f.addr(h + 8 + 2 * f.sl);
    int budget = 4096;
    walk_btree(f, btree, heap_data, out, 0, budget);
    std::stable_sort(out.begin(), out.end(), [](const Entry &a, const Entry &b) {
        return strcmp(a.name.c_str(), b.name.c_str()) < 0;
    });
    return true;
}

bool is_dataset(const File &f, uint64_t oh) { return find(object_messages(f, oh), 0x08) != nullptr; }

// A float dataset's shape and where its values are.
struct DsInfo {
    std::vector<uint64_t> dims;
    uint64_t count = 1, data_off = 0;
    uint32_t esz = 4;
    bool be = false, undefined = false;
};

DsInfo dataset_info(const File &f, uint64_t oh) {
    auto ms = object_messages(f, oh);
    const Msg *sp = find(ms, 0x01), *ty = find(ms, 0x03), *lay = find(ms, 0x08);
    if (!sp || !ty || !lay) fail(NR_E_FORMAT, "HDF5: dataset lacks dataspace/datatype/layout");
    if (ty->flags & 0x02) fail(NR_E_FORMAT, "HDF5: shared (committed) datatypes unsupported");
    if (find(ms, 0x0B)) fail(NR_E_FORMAT, "HDF5: filtered datasets unsupported");
    DsInfo I;
    // dataspace (every field read through a bounds-checked accessor: a message may be shorter than
    // its type's layout in a damaged file)
    int sv = f.byte(sp->off), nd = f.byte(sp->off + 1);
    uint64_t dp = (sv == 1) ? sp->off + 8 : (sv == 2 ? sp->off + 4 : 0);
    if (!dp) fail(NR_E_FORMAT, "HDF5: unknown dataspace version");
    I.dims.resize(nd);
    for (int i = 0; i < nd; ++i) {
        I.dims[i] = f.uint(dp + (uint64_t)i * f.sl, f.sl);
        // no product past 2^31 elements (a file is at most 1 GiB): the byte count cannot wrap
        if (I.dims[i] > (1ull << 31) || (I.count *= I.dims[i]) > (1ull << 31)) fail(NR_E_FORMAT, "HDF5: dataset too large");
    }
    // datatype
    int cls = f.byte(ty->off) & 0x0f;
    uint8_t bits0 = f.byte(ty->off + 1);
    I.esz = (uint32_t)f.uint(ty->off + 4, 4);
    if (cls != 1 || (I.esz != 4 && I.esz != 8)) fail(NR_E_FORMAT, "HDF5: dataset is not IEEE float32/float64");
    I.be = bits0 & 1;
    // layout
    int lv = f.byte(lay->off);
    const uint64_t data_len = I.count * I.esz;
    if (lv == 3 || lv == 4) {
        int lc = f.byte(lay->off + 1);
        if (lc == 1) {
            uint64_t a = f.addr(lay->off + 2);
            I.undefined = f.undef(a);
            I.data_off = f.abs(a);
        } else if (lc == 0) {
            uint64_t n = f.uint(lay->off + 2, 2);
            if (n < data_len) fail(NR_E_FORMAT, "HDF5: compact dataset too small");
            I.data_off = lay->off + 4;
        } else {
            fail(NR_E_FORMAT, "HDF5: chunked/virtual datasets unsupported");
        }
    } else if (lv == 1 || lv == 2) {
        int lnd = f.byte(lay->off + 1), lc = f.byte(lay->off + 2);
        if (lc == 1) {
            uint64_t a = f.addr(lay->off + 8);
            I.undefined = f.undef(a);
            I.data_off = f.abs(a);
        } else if (lc == 0) {
            I.data_off = lay->off + 8 + (uint64_t)lnd * 4 + 4;
        } else {
            fail(NR_E_FORMAT, "HDF5: chunked datasets unsupported");
        }
    } else {
        fail(NR_E_FORMAT, "HDF5: unknown layout message version");
    }
    if (!I.undefined) f.need(I.data_off, data_len);
    return I;
}

// Reads a float dataset's values (as float) into out[0, count); returns its dims.
void read_values(const File &f, const DsInfo &I, float *out) {
    if (I.undefined) {  // never written: fill value 0
        std::fill(out, out + I.count, 0.0f);
        return;
    }
    for (uint64_t i = 0; i < I.count; ++i) {
        uint8_t b[8];
        memcpy(b, &f.d[I.data_off + i * I.esz], I.esz);
        if (I.be) std::reverse(b, b + I.esz);
        if (I.esz == 4) { float v; memcpy(&v, b, 4); out[i] = v; }
        else { double v; memcpy(&v, b, 8); out[i] = (float)v; }
    }
}

std::vector<uint64_t> read_dataset(const File &f, uint64_t oh, std::vector<float> &vals) {
    const DsInfo I = dataset_info(f, oh);
    vals.assign(I.count, 0.0f);
    read_values(f, I, vals.data());
    return I.dims;
}

void open_file(const char *path, File &f) {
    FILE *fp = fopen(path, "rb");
    if (!fp) fail(NR_E_IO, std::string("cannot open ") + path);
    fseek(fp, 0, SEEK_END);
    long n = ftell(fp);
    fseek(fp, 0, SEEK_SET);
    if (n <= 0 || n > (1l << 30)) { fclose(fp); fail(NR_E_FORMAT, "HDF5: bad file size"); }
    f.d.resize((size_t)n);
    size_t got = fread(f.d.data(), 1, (size_t)n, fp);
    fclose(fp);
    if (got != (size_t)n) fail(NR_E_IO, "short read");
    static const uint8_t sig[8] = {0x89, 'H', 'D', 'F', '\r', '\n', 0x1a, '\n'};
    uint64_t sb = ~0ull;
    for (uint64_t o = 0; o + 8 <= f.d.size(); o = o ? o * 2 : 512) {
        if (memcmp(&f.d[o], sig, 8) == 0) { sb = o; break; }
        if (o > (1u << 24)) break;
    }
    if (sb == ~0ull) fail(NR_E_FORMAT, "not an HDF5 file");
    f.sb = sb;
    int ver = f.byte(sb + 8);
    if (ver > 1) fail(NR_E_FORMAT, "HDF5: superblock version >1 unsupported");
    f.so = f.byte(sb + 13);
    f.sl = f.byte(sb + 14);
    if ((f.so != 2 && f.so != 4 && f.so != 8) || (f.sl != 2 && f.sl != 4 && f.sl != 8))
        fail(NR_E_FORMAT, "HDF5: bad offset/length sizes in the superblock");
    if ((f.so != 4 && f.so != 8) || (f.sl != 4 && f.sl != 8)) fail(NR_E_FORMAT, "HDF5: odd offset size");
    uint64_t p = sb + 24 + (ver == 1 ? 4 : 0);
    f.base = f.addr(p);
    if (f.base == 0) f.base = sb;
}

uint64_t root_object(const File &f) {
    // the root symbol-table entry follows the 4 addresses of the superblock
    const int ver = f.byte(f.sb + 8);
    const uint64_t rootent = f.sb + 24 + (ver == 1 ? 4 : 0) + 4 * (uint64_t)f.so;
    return f.addr(rootent + f.so);
}

}  // namespace

// Reads a Keras Dense stack the way NeuralNetwork::load does (neuralNetwork.cpp:85-151).
int h5_read_keras(const char *path, std::vector<int> &dims, std::vector<std::vector<float>> &kernels,
                  std::vector<std::vector<float>> &biases, std::string &err) {
    try {
        File f;
        open_file(path, f);
        const uint64_t root_oh = root_object(f);
        std::vector<Entry> layers;
        if (!group_members(f, root_oh, layers)) fail(NR_E_FORMAT, "HDF5: root is not a group");
        dims.clear(); kernels.clear(); biases.clear();
        for (auto &L : layers) {
            std::vector<Entry> inner;
            if (!group_members(f, L.oh, inner)) fail(NR_E_FORMAT, "Unsupported Layer");  // :93-96
            if (inner.size() != 1) fail(NR_E_FORMAT, "Unsupported Layer");              // :101-104
            if (inner[0].name != L.name) fail(NR_E_FORMAT, "Unsupported Layer: inner group name mismatch");
            std::vector<Entry> mats;
            if (!group_members(f, inner[0].oh, mats)) fail(NR_E_FORMAT, "Unsupported Layer");
            std::vector<float> W, b;
            std::vector<uint64_t> wd;
            bool haveW = false, haveB = false;
            for (auto &m : mats) {
                if (!is_dataset(f, m.oh)) fail(NR_E_FORMAT, "Unsupported Layer");     // :116-119
                std::vector<float> v;
                auto d = read_dataset(f, m.oh, v);
                if (d.size() == 1) { b = v; haveB = true; }
                else if (d.size() == 2) { W = v; wd = d; haveW = true; }
                else fail(NR_E_FORMAT, "Unsupported layer, to many dims!");          // :127-130
            }
            if (!haveW || !haveB) fail(NR_E_FORMAT, "Unsupported Layer: missing kernel or bias");
            int in = (int)wd[0], out = (int)wd[1];
            if ((int)b.size() != out) fail(NR_E_FORMAT, "Unsupported Layer: bias size != kernel columns");
            if (dims.empty()) dims.push_back(in);
            else if (dims.back() != in) fail(NR_E_FORMAT, "Unsupported Layer: layer input size mismatch");
            dims.push_back(out);
            kernels.push_back(std::move(W));
            biases.push_back(std::move(b));
        }
        if (kernels.empty()) fail(NR_E_FORMAT, "HDF5: no layers found");
        return NR_OK;
    } catch (const H5Error &e) {
        err = e.msg;
        return e.code;
    }
}

}  // namespace nr

// ---- HDF5 object tree (C ABI, neural_render.h nr_h5_*): what the HighFive subset in
// include/highfive/ wraps.  Objects are named by their object-header addresses.
struct nr_h5_file {
    nr::File f;
    uint64_t root = 0;
    std::map<uint64_t, std::vector<nr::Entry>> members;  // group -> members, name order
};

namespace {
const std::vector<nr::Entry> &members_of(nr_h5_file *h, uint64_t g) {
    auto it = h->members.find(g);
    if (it != h->members.end()) return it->second;
    std::vector<nr::Entry> m;
    if (!nr::group_members(h->f, g, m)) nr::fail(NR_E_INVALID, "HDF5: object is not a group");
    return h->members.emplace(g, std::move(m)).first->second;
}
}  // namespace

extern "C" {

int nr_h5_open(const char *path, nr_h5_file **out) {
    if (!path || !out) return nr::report_error(NR_E_INVALID, "nr_h5_open: NULL argument");
    *out = nullptr;
    nr_h5_file *h = new (std::nothrow) nr_h5_file;
    if (!h) return nr::report_error(NR_E_NOMEM, "out of host memory");
    try {
        nr::open_file(path, h->f);
        h->root = nr::root_object(h->f);
        members_of(h, h->root);  // the root must be a symbol-table group
    } catch (const nr::H5Error &e) {
        delete h;
        return nr::report_error(e.code, "%s", e.msg.c_str());
    }
    *out = h;
    return NR_OK;
}

void nr_h5_close(nr_h5_file *h) { delete h; }

int nr_h5_root(const nr_h5_file *h, uint64_t *obj) {
    if (!h || !obj) return nr::report_error(NR_E_INVALID, "nr_h5_root: NULL argument");
    *obj = h->root;
    return NR_OK;
}

int nr_h5_object_type(nr_h5_file *h, uint64_t obj, int *type) {
    if (!h || !type) return nr::report_error(NR_E_INVALID, "nr_h5_object_type: NULL argument");
    try {
        const auto ms = nr::object_messages(h->f, obj);
        *type = nr::find(ms, 0x11) ? NR_H5_GROUP : (nr::find(ms, 0x08) ? NR_H5_DATASET : NR_H5_OTHER);
    } catch (const nr::H5Error &e) {
        return nr::report_error(e.code, "%s", e.msg.c_str());
    }
    return NR_OK;
}

int nr_h5_num_members(nr_h5_file *h, uint64_t group, size_t *n) {
    if (!h || !n) return nr::report_error(NR_E_INVALID, "nr_h5_num_members: NULL argument");
    try {
        *n = members_of(h, group).size();
    } catch (const nr::H5Error &e) {
        return nr::report_error(e.code, "%s", e.msg.c_str());
    }
    return NR_OK;
}

int nr_h5_member(nr_h5_file *h, uint64_t group, size_t i, char *name, size_t cap, size_t *name_len, uint64_t *obj) {
    if (!h) return nr::report_error(NR_E_INVALID, "nr_h5_member: NULL file");
    try {
        const auto &m = members_of(h, group);
        if (i >= m.size()) return nr::report_error(NR_E_INVALID, "nr_h5_member: index %zu of %zu members", i, m.size());
        if (name_len) *name_len = m[i].name.size();
        if (obj) *obj = m[i].oh;
        if (name) {
            if (cap < m[i].name.size() + 1) return nr::report_error(NR_E_INVALID, "nr_h5_member: name buffer too small");
            memcpy(name, m[i].name.c_str(), m[i].name.size() + 1);
        }
    } catch (const nr::H5Error &e) {
        return nr::report_error(e.code, "%s", e.msg.c_str());
    }
    return NR_OK;
}

int nr_h5_dims(nr_h5_file *h, uint64_t dataset, uint64_t *dims, int cap, int *ndims) {
    if (!h || !ndims) return nr::report_error(NR_E_INVALID, "nr_h5_dims: NULL argument");
    try {
        const nr::DsInfo I = nr::dataset_info(h->f, dataset);
        *ndims = (int)I.dims.size();
        if (dims) {
            if (cap < (int)I.dims.size()) return nr::report_error(NR_E_INVALID, "nr_h5_dims: dims buffer too small");
            for (size_t k = 0; k < I.dims.size(); ++k) dims[k] = I.dims[k];
        }
    } catch (const nr::H5Error &e) {
        return nr::report_error(e.code, "%s", e.msg.c_str());
    }
    return NR_OK;
}

int nr_h5_read_f32(nr_h5_file *h, uint64_t dataset, float *out, size_t count) {
    if (!h || (count && !out)) return nr::report_error(NR_E_INVALID, "nr_h5_read_f32: NULL argument");
    try {
        const nr::DsInfo I = nr::dataset_info(h->f, dataset);
        if (count != I.count)
            return nr::report_error(NR_E_INVALID, "nr_h5_read_f32: dataset has %llu elements, buffer %zu",
                                    (unsigned long long)I.count, count);
        nr::read_values(h->f, I, out);
    } catch (const nr::H5Error &e) {
        return nr::report_error(e.code, "%s", e.msg.c_str());
    }
    return NR_OK;
}

}  // extern "C"
