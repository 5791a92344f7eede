// Native HDF5 I/O for the Level-1 / Level-2 wire format (include/comap_h5.h).
//
// The reference reads and writes its files through h5py
// (comancpipeline/Analysis/DataHandling.py:101-179, MapMaking/COMAPData.py:170,
// 252, 389, 435).  This is the same file layer on the HDF5 C library: a visit of
// every object below the root, typed whole / hyperslab / flat-range reads, and
// writes that create intermediate groups and replace existing objects.  Types
// follow h5py's mapping (bool = int8 enum {FALSE, TRUE}, str = variable-length
// UTF-8, bytes = fixed-length NULLPAD) so either side reads the other's files.
//
// Host code only: the Level-1 cube is read in flat element ranges straight into
// the caller's (pinned) staging buffers, which gpu.upload drains to the device.
#include <fcntl.h>
#include <hdf5.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <cerrno>
#include <cstdint>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#include "../../include/comap_h5.h"

struct comap_h5 {
    hid_t file = -1;
    bool readonly = false;
    std::string path;
    int fd = -1;              // POSIX descriptor for the direct read path (opened on first use)
};

namespace {

thread_local std::string g_err;

struct Init {
    Init() { H5Eset_auto2(H5E_DEFAULT, nullptr, nullptr); }   // errors are returned, not printed
} g_init;

herr_t err_walk(unsigned n, const H5E_error2_t *e, void *data)
{
    auto *s = static_cast<std::string *>(data);
    if (n == 0 && e && e->desc) *s = e->desc;                  // innermost description
    return 0;
}

int fail(const std::string &what, int code = -2)
{
    std::string inner;
    H5Ewalk2(H5E_DEFAULT, H5E_WALK_DOWNWARD, err_walk, &inner);
    H5Eclear2(H5E_DEFAULT);
    g_err = inner.empty() ? what : what + ": " + inner;
    return code;
}

// closes an HDF5 identifier of any kind on scope exit
struct Hid {
    hid_t id = -1;
    Hid() = default;
    explicit Hid(hid_t h) : id(h) {}
    Hid(const Hid &) = delete;
    Hid &operator=(const Hid &) = delete;
    ~Hid() { reset(); }
    void reset(hid_t h = -1)
    {
        if (id >= 0) {
            switch (H5Iget_type(id)) {
            case H5I_FILE: H5Fclose(id); break;
            case H5I_GROUP: H5Gclose(id); break;
            case H5I_DATASET: H5Dclose(id); break;
            case H5I_DATASPACE: H5Sclose(id); break;
            case H5I_DATATYPE: H5Tclose(id); break;
            case H5I_ATTR: H5Aclose(id); break;
            case H5I_GENPROP_LST: H5Pclose(id); break;
            default: break;
            }
        }
        id = h;
    }
    operator hid_t() const { return id; }
    bool ok() const { return id >= 0; }
};

std::string norm(const char *path)
{
    std::string p = path ? path : "";
    while (!p.empty() && p.back() == '/') p.pop_back();
    return p.empty() ? std::string("/") : p;
}

// every link along path exists (H5Lexists needs its parents to exist)
bool path_exists(hid_t file, const std::string &p)
{
    if (p == "/") return true;
    size_t pos = p[0] == '/' ? 1 : 0;
    while (true) {
        const size_t next = p.find('/', pos);
        const std::string sub = p.substr(0, next);
        if (H5Lexists(file, sub.c_str(), H5P_DEFAULT) <= 0) return false;
        if (next == std::string::npos) break;
        pos = next + 1;
    }
    return H5Oexists_by_name(file, p.c_str(), H5P_DEFAULT) > 0;
}

hid_t bool_type()
{
    const hid_t t = H5Tenum_create(H5T_NATIVE_INT8);
    int8_t v = 0;
    H5Tenum_insert(t, "FALSE", &v);
    v = 1;
    H5Tenum_insert(t, "TRUE", &v);
    return t;
}

// in-memory (and on-file, for writes) type of a dtype code
hid_t mem_type(int32_t dtype, int64_t elsize)
{
    switch (dtype) {
    case COMAP_H5_F32: return H5Tcopy(H5T_NATIVE_FLOAT);
    case COMAP_H5_F64: return H5Tcopy(H5T_NATIVE_DOUBLE);
    case COMAP_H5_I8: return H5Tcopy(H5T_NATIVE_INT8);
    case COMAP_H5_I16: return H5Tcopy(H5T_NATIVE_INT16);
    case COMAP_H5_I32: return H5Tcopy(H5T_NATIVE_INT32);
    case COMAP_H5_I64: return H5Tcopy(H5T_NATIVE_INT64);
    case COMAP_H5_U8: return H5Tcopy(H5T_NATIVE_UINT8);
    case COMAP_H5_U16: return H5Tcopy(H5T_NATIVE_UINT16);
    case COMAP_H5_U32: return H5Tcopy(H5T_NATIVE_UINT32);
    case COMAP_H5_U64: return H5Tcopy(H5T_NATIVE_UINT64);
    case COMAP_H5_BOOL: return bool_type();
    case COMAP_H5_STR_FIXED: {
        if (elsize < 1) return -1;
        const hid_t t = H5Tcopy(H5T_C_S1);
        H5Tset_size(t, (size_t)elsize);
        H5Tset_strpad(t, H5T_STR_NULLPAD);
        return t;
    }
    case COMAP_H5_STR_VLEN: {
        const hid_t t = H5Tcopy(H5T_C_S1);
        H5Tset_size(t, H5T_VARIABLE);
        H5Tset_cset(t, H5T_CSET_UTF8);
        return t;
    }
    default: return -1;
    }
}

int32_t classify(hid_t t, int64_t *elsize)
{
    const size_t sz = H5Tget_size(t);
    *elsize = (int64_t)sz;
    switch (H5Tget_class(t)) {
    case H5T_FLOAT: return sz == 4 ? COMAP_H5_F32 : sz == 8 ? COMAP_H5_F64 : COMAP_H5_UNSUPPORTED;
    case H5T_INTEGER: {
        const bool sgn = H5Tget_sign(t) == H5T_SGN_2;
        switch (sz) {
        case 1: return sgn ? COMAP_H5_I8 : COMAP_H5_U8;
        case 2: return sgn ? COMAP_H5_I16 : COMAP_H5_U16;
        case 4: return sgn ? COMAP_H5_I32 : COMAP_H5_U32;
        case 8: return sgn ? COMAP_H5_I64 : COMAP_H5_U64;
        default: return COMAP_H5_UNSUPPORTED;
        }
    }
    case H5T_ENUM: {
        if (H5Tget_nmembers(t) == 2 && sz == 1) {
            char *a = H5Tget_member_name(t, 0), *b = H5Tget_member_name(t, 1);
            const bool isbool = a && b && ((!strcmp(a, "FALSE") && !strcmp(b, "TRUE")) ||
                                           (!strcmp(a, "TRUE") && !strcmp(b, "FALSE")));
            H5free_memory(a);
            H5free_memory(b);
            if (isbool) return COMAP_H5_BOOL;
        }
        Hid base(H5Tget_super(t));
        return base.ok() ? classify(base, elsize) : COMAP_H5_UNSUPPORTED;
    }
    case H5T_STRING:
        if (H5Tis_variable_str(t) > 0) {
            *elsize = (int64_t)sizeof(char *);
            return COMAP_H5_STR_VLEN;
        }
        return COMAP_H5_STR_FIXED;
    default: return COMAP_H5_UNSUPPORTED;
    }
}

int space_shape(hid_t space, int32_t *ndim, int64_t *dims)
{
    const int nd = H5Sget_simple_extent_ndims(space);
    if (nd < 0 || nd > COMAP_H5_MAX_RANK) return fail("dataspace rank");
    hsize_t d[COMAP_H5_MAX_RANK];
    if (nd > 0 && H5Sget_simple_extent_dims(space, d, nullptr) < 0) return fail("dataspace dims");
    *ndim = nd;
    for (int i = 0; i < nd; ++i) dims[i] = (int64_t)d[i];
    return 0;
}

// select the flat row-major element range [off, off + n) of a dataspace of dims[nd]
// as a union of at most 2 nd - 1 hyperslabs (HDF5 transfers the selected elements
// in row-major file order, whatever order they were added in)
herr_t select_flat(hid_t space, const hsize_t *dims, int nd, hsize_t off, hsize_t n, hsize_t *start, hsize_t *count,
                   int depth)
{
    if (n == 0) return 0;
    hsize_t inner = 1;
    for (int i = depth + 1; i < nd; ++i) inner *= dims[i];
    if (depth == nd - 1) {                     // a run along the last axis
        start[depth] = off;
        count[depth] = n;
        return H5Sselect_hyperslab(space, H5S_SELECT_OR, start, nullptr, count, nullptr);
    }
    hsize_t i0 = off / inner, r0 = off % inner;
    if (r0) {                                  // head: the rest of slab i0
        const hsize_t m = n < inner - r0 ? n : inner - r0;
        start[depth] = i0;
        count[depth] = 1;
        if (select_flat(space, dims, nd, r0, m, start, count, depth + 1) < 0) return -1;
        n -= m;
        ++i0;
    }
    const hsize_t full = n / inner;
    if (full) {                                // whole slabs
        start[depth] = i0;
        count[depth] = full;
        for (int i = depth + 1; i < nd; ++i) { start[i] = 0; count[i] = dims[i]; }
        if (H5Sselect_hyperslab(space, H5S_SELECT_OR, start, nullptr, count, nullptr) < 0) return -1;
        i0 += full;
        n -= full * inner;
    }
    if (n) {                                   // tail: the start of slab i0
        start[depth] = i0;
        count[depth] = 1;
        if (select_flat(space, dims, nd, 0, n, start, count, depth + 1) < 0) return -1;
    }
    return 0;
}

int64_t put_text(const std::string &s, char *buf, int64_t cap)
{
    if (buf && cap > 0) {
        const size_t m = std::min<size_t>((size_t)cap - 1, s.size());
        memcpy(buf, s.data(), m);
        buf[m] = '\0';
    }
    return (int64_t)s.size() + 1;
}

struct VisitState {
    std::string out;
};

herr_t visit_cb(hid_t g, const char *name, const H5L_info_t *info, void *data)
{
    if (info->type != H5L_TYPE_HARD) return 0;   // soft / external links: not followed
    Hid o(H5Oopen(g, name, H5P_DEFAULT));
    if (!o.ok()) return 0;
    const H5I_type_t t = H5Iget_type(o);
    auto *st = static_cast<VisitState *>(data);
    if (t == H5I_DATASET || t == H5I_GROUP) {
        st->out += t == H5I_DATASET ? "D " : "G ";
        st->out += name;
        st->out += '\n';
    }
    return 0;
}

herr_t attr_cb(hid_t, const char *name, const H5A_info_t *, void *data)
{
    auto *s = static_cast<std::string *>(data);
    *s += name;
    *s += '\n';
    return 0;
}

int make_space(int32_t ndim, const int64_t *dims, Hid &space)
{
    if (ndim < 0 || ndim > COMAP_H5_MAX_RANK) return fail("rank out of range", -1);
    if (ndim == 0) {
        space.reset(H5Screate(H5S_SCALAR));
    } else {
        hsize_t d[COMAP_H5_MAX_RANK];
        for (int i = 0; i < ndim; ++i) {
            if (dims[i] < 0) return fail("negative dimension", -1);
            d[i] = (hsize_t)dims[i];
        }
        space.reset(H5Screate_simple(ndim, d, nullptr));
    }
    return space.ok() ? 0 : fail("H5Screate");
}

int64_t n_elements(int32_t ndim, const int64_t *dims)
{
    int64_t n = 1;
    for (int i = 0; i < ndim; ++i) n *= dims[i];
    return n;
}

// strings of an attribute or dataset of variable-length strings, back to back
int64_t read_vlen(hid_t obj, bool is_attr, char *buf, int64_t cap)
{
    Hid space(is_attr ? H5Aget_space(obj) : H5Dget_space(obj));
    if (!space.ok()) return fail("get_space");
    const hssize_t n = H5Sget_simple_extent_npoints(space);
    if (n < 0) return fail("npoints");
    Hid mt(mem_type(COMAP_H5_STR_VLEN, 0));
    std::vector<char *> ptr((size_t)n + 1, nullptr);
    const herr_t e = is_attr ? H5Aread(obj, mt, ptr.data()) : H5Dread(obj, mt, H5S_ALL, H5S_ALL, H5P_DEFAULT, ptr.data());
    if (e < 0) return fail("read variable-length strings");
    std::string out;
    for (hssize_t i = 0; i < n; ++i) {
        if (ptr[i]) out += ptr[i];
        out += '\0';
    }
    H5Dvlen_reclaim(mt, space, H5P_DEFAULT, ptr.data());
    if (buf && cap >= (int64_t)out.size()) memcpy(buf, out.data(), out.size());
    return (int64_t)out.size();
}

std::vector<const char *> split_strings(const char *buf, int64_t n)
{
    std::vector<const char *> v((size_t)n);
    const char *p = buf;
    for (int64_t i = 0; i < n; ++i) {
        v[(size_t)i] = p;
        p += strlen(p) + 1;
    }
    return v;
}

bool valid(const comap_h5 *f) { return f && f->file >= 0; }

// Direct path of comap_h5_read_flat: a contiguous (unchunked, unfiltered) dataset
// whose stored type is the requested native little-endian type is one byte range of
// the file (H5Dget_offset), so a flat element range is read with pread by several
// threads at once -- HDF5 itself is not thread-safe, and one H5Dread memcpy thread
// is what bounds a page-cache-hot cube's staging rate.  Read-only files only (no
// unflushed library buffers).  Returns 1 when it handled the read, 0 to fall back.
constexpr int64_t kDirectMinBytes = 8ll << 20;     // below this one H5Dread is as fast
constexpr int64_t kDirectPerThread = 32ll << 20;

int direct_read(comap_h5 *f, hid_t d, hid_t ftype, hid_t mtype, int64_t elsize, int64_t offset, int64_t n, void *buf,
                std::string *err)
{
    if (!f->readonly || n * elsize < kDirectMinBytes) return 0;
    Hid dcpl(H5Dget_create_plist(d));
    if (!dcpl.ok() || H5Pget_layout(dcpl) != H5D_CONTIGUOUS || H5Pget_nfilters(dcpl) != 0) return 0;
    if (H5Tequal(ftype, mtype) <= 0 || H5Tget_order(ftype) != H5T_ORDER_LE) return 0;
    const haddr_t base = H5Dget_offset(d);
    if (base == HADDR_UNDEF) return 0;
    if (f->fd < 0) {
        f->fd = ::open(f->path.c_str(), O_RDONLY | O_CLOEXEC);
        if (f->fd < 0) return 0;
    }
    const int64_t bytes = n * elsize;
    const int64_t start = (int64_t)base + offset * elsize;
    const unsigned hw = std::max(1u, std::thread::hardware_concurrency());
    const int nt = (int)std::max<int64_t>(1, std::min<int64_t>({(int64_t)16, (int64_t)hw, bytes / kDirectPerThread}));
    const int64_t per = (bytes + nt - 1) / nt;
    // errno is per thread and a short read sets none: each worker records its own
    // failure (errno, or the file offset of an unexpected end of file)
    std::vector<int> eno(nt, 0);
    std::vector<int64_t> short_at(nt, -1);
    auto work = [&](int i) {
        int64_t lo = (int64_t)i * per, hi = std::min(bytes, lo + per);
        char *dst = static_cast<char *>(buf);
        while (lo < hi) {
            const ssize_t r = ::pread(f->fd, dst + lo, (size_t)std::min<int64_t>(hi - lo, 1ll << 30), start + lo);
            if (r < 0 && errno == EINTR) continue;
            if (r < 0) { eno[i] = errno; return; }
            if (r == 0) { short_at[i] = start + lo; return; }
            lo += r;
        }
    };
    std::vector<std::thread> th;
    for (int i = 1; i < nt; ++i) th.emplace_back(work, i);
    work(0);
    for (auto &t : th) t.join();
    for (int i = 0; i < nt; ++i) {
        if (eno[i]) { *err = strerror(eno[i]); return -1; }
        if (short_at[i] >= 0) { *err = "short read (end of file) at byte offset " + std::to_string(short_at[i]); return -1; }
    }
    return 1;
}

}  // namespace

extern "C" {

const char *comap_h5_version(void)
{
    static std::string v;
    if (v.empty()) {
        unsigned a = 0, b = 0, c = 0;
        H5get_libversion(&a, &b, &c);
        v = "comap_h5 (HDF5 " + std::to_string(a) + "." + std::to_string(b) + "." + std::to_string(c) + ")";
    }
    return v.c_str();
}

const char *comap_h5_last_error(void) { return g_err.c_str(); }

int comap_h5_open(const char *path, int32_t mode, comap_h5 **out)
{
    if (!path || !out) return fail("comap_h5_open: bad arguments", -1);
    *out = nullptr;
    hid_t f = -1;
    if (mode == 0) {
        f = H5Fopen(path, H5F_ACC_RDONLY, H5P_DEFAULT);
    } else if (mode == 1) {
        const htri_t is = H5Fis_hdf5(path);
        f = is > 0 ? H5Fopen(path, H5F_ACC_RDWR, H5P_DEFAULT) : H5Fcreate(path, H5F_ACC_EXCL, H5P_DEFAULT, H5P_DEFAULT);
    } else if (mode == 2) {
        f = H5Fcreate(path, H5F_ACC_TRUNC, H5P_DEFAULT, H5P_DEFAULT);
    } else {
        return fail("comap_h5_open: mode must be 0, 1 or 2", -1);
    }
    if (f < 0) return fail(std::string("cannot open ") + path);
    *out = new comap_h5;
    (*out)->file = f;
    (*out)->readonly = mode == 0;
    (*out)->path = path;
    return 0;
}

int comap_h5_close(comap_h5 *f)
{
    if (!f) return 0;
    int rc = 0;
    if (f->fd >= 0) ::close(f->fd);
    if (f->file >= 0 && H5Fclose(f->file) < 0) rc = fail("H5Fclose");
    delete f;
    return rc;
}

int comap_h5_flush(comap_h5 *f)
{
    if (!valid(f)) return fail("comap_h5_flush: closed file", -1);
    return H5Fflush(f->file, H5F_SCOPE_LOCAL) < 0 ? fail("H5Fflush") : 0;
}

int comap_h5_exists(comap_h5 *f, const char *path)
{
    if (!valid(f) || !path) return fail("comap_h5_exists: bad arguments", -1);
    return path_exists(f->file, norm(path)) ? 1 : 0;
}

int64_t comap_h5_visit(comap_h5 *f, char *buf, int64_t cap)
{
    if (!valid(f)) return fail("comap_h5_visit: closed file", -1);
    VisitState st;
    if (H5Lvisit(f->file, H5_INDEX_NAME, H5_ITER_INC, visit_cb, &st) < 0) return fail("H5Lvisit");
    return put_text(st.out, buf, cap);
}

int comap_h5_require_group(comap_h5 *f, const char *path)
{
    if (!valid(f) || !path) return fail("comap_h5_require_group: bad arguments", -1);
    const std::string p = norm(path);
    if (path_exists(f->file, p)) {
        Hid o(H5Oopen(f->file, p.c_str(), H5P_DEFAULT));
        if (!o.ok() || H5Iget_type(o) != H5I_GROUP) return fail(p + " exists and is not a group", -1);
        return 0;
    }
    Hid lcpl(H5Pcreate(H5P_LINK_CREATE));
    H5Pset_create_intermediate_group(lcpl, 1);
    Hid g(H5Gcreate2(f->file, p.c_str(), lcpl, H5P_DEFAULT, H5P_DEFAULT));
    return g.ok() ? 0 : fail("create group " + p);
}

int comap_h5_delete(comap_h5 *f, const char *path)
{
    if (!valid(f) || !path) return fail("comap_h5_delete: bad arguments", -1);
    const std::string p = norm(path);
    if (!path_exists(f->file, p)) return 0;
    return H5Ldelete(f->file, p.c_str(), H5P_DEFAULT) < 0 ? fail("delete " + p) : 0;
}

int comap_h5_info(comap_h5 *f, const char *path, int32_t *dtype, int32_t *ndim, int64_t *dims, int64_t *elsize)
{
    if (!valid(f) || !path || !dtype || !ndim || !dims || !elsize) return fail("comap_h5_info: bad arguments", -1);
    Hid d(H5Dopen2(f->file, norm(path).c_str(), H5P_DEFAULT));
    if (!d.ok()) return fail(std::string("no dataset ") + path, -3);
    Hid t(H5Dget_type(d)), s(H5Dget_space(d));
    if (!t.ok() || !s.ok()) return fail("dataset type/space");
    *dtype = classify(t, elsize);
    return space_shape(s, ndim, dims);
}

int comap_h5_read(comap_h5 *f, const char *path, int32_t dtype, int64_t elsize, const int64_t *start,
                  const int64_t *count, void *buf)
{
    if (!valid(f) || !path) return fail("comap_h5_read: bad arguments", -1);
    Hid d(H5Dopen2(f->file, norm(path).c_str(), H5P_DEFAULT));
    if (!d.ok()) return fail(std::string("no dataset ") + path, -3);
    Hid mt(mem_type(dtype, elsize));
    if (!mt.ok() || dtype == COMAP_H5_STR_VLEN) return fail("comap_h5_read: unsupported dtype", -1);
    Hid fs(H5Dget_space(d));
    int32_t nd = 0;
    int64_t dims[COMAP_H5_MAX_RANK];
    if (space_shape(fs, &nd, dims)) return -2;
    if (!start || !count || nd == 0) {
        if (n_elements(nd, dims) == 0) return 0;
        if (!buf) return fail("comap_h5_read: no buffer", -1);
        return H5Dread(d, mt, H5S_ALL, H5S_ALL, H5P_DEFAULT, buf) < 0 ? fail(std::string("read ") + path) : 0;
    }
    hsize_t st[COMAP_H5_MAX_RANK], ct[COMAP_H5_MAX_RANK];
    hsize_t total = 1;
    for (int i = 0; i < nd; ++i) {
        if (start[i] < 0 || count[i] < 0 || start[i] + count[i] > dims[i])
            return fail(std::string("hyperslab out of range in ") + path, -1);
        st[i] = (hsize_t)start[i];
        ct[i] = (hsize_t)count[i];
        total *= ct[i];
    }
    if (total == 0) return 0;
    if (!buf) return fail("comap_h5_read: no buffer", -1);
    if (H5Sselect_hyperslab(fs, H5S_SELECT_SET, st, nullptr, ct, nullptr) < 0) return fail("select hyperslab");
    Hid ms(H5Screate_simple(1, &total, nullptr));
    return H5Dread(d, mt, ms, fs, H5P_DEFAULT, buf) < 0 ? fail(std::string("read ") + path) : 0;
}

int comap_h5_read_flat(comap_h5 *f, const char *path, int32_t dtype, int64_t elsize, int64_t offset, int64_t n,
                       void *buf)
{
    if (!valid(f) || !path || offset < 0 || n < 0) return fail("comap_h5_read_flat: bad arguments", -1);
    if (n == 0) return 0;
    if (!buf) return fail("comap_h5_read_flat: no buffer", -1);
    Hid d(H5Dopen2(f->file, norm(path).c_str(), H5P_DEFAULT));
    if (!d.ok()) return fail(std::string("no dataset ") + path, -3);
    Hid mt(mem_type(dtype, elsize));
    if (!mt.ok() || dtype == COMAP_H5_STR_VLEN) return fail("comap_h5_read_flat: unsupported dtype", -1);
    Hid fs(H5Dget_space(d));
    int32_t nd = 0;
    int64_t dims[COMAP_H5_MAX_RANK];
    if (space_shape(fs, &nd, dims)) return -2;
    if (offset + n > n_elements(nd, dims)) return fail(std::string("flat range out of range in ") + path, -1);
    {
        Hid ft(H5Dget_type(d));
        std::string err;
        const int dr = ft.ok() ? direct_read(f, d, ft, mt, elsize, offset, n, buf, &err) : 0;
        if (dr < 0) return fail(std::string("pread ") + f->path + ": " + err);
        if (dr > 0) return 0;
    }
    if (nd == 0) return H5Dread(d, mt, H5S_ALL, H5S_ALL, H5P_DEFAULT, buf) < 0 ? fail("read scalar") : 0;
    hsize_t hd[COMAP_H5_MAX_RANK], st[COMAP_H5_MAX_RANK] = {0}, ct[COMAP_H5_MAX_RANK] = {0};
    for (int i = 0; i < nd; ++i) { hd[i] = (hsize_t)dims[i]; ct[i] = 1; }
    if (H5Sselect_none(fs) < 0 || select_flat(fs, hd, nd, (hsize_t)offset, (hsize_t)n, st, ct, 0) < 0)
        return fail("select flat range");
    const hsize_t m = (hsize_t)n;
    Hid ms(H5Screate_simple(1, &m, nullptr));
    return H5Dread(d, mt, ms, fs, H5P_DEFAULT, buf) < 0 ? fail(std::string("read ") + path) : 0;
}

int comap_h5_write(comap_h5 *f, const char *path, int32_t dtype, int64_t elsize, int32_t ndim, const int64_t *dims,
                   const void *buf)
{
    if (!valid(f) || !path || (ndim > 0 && !dims)) return fail("comap_h5_write: bad arguments", -1);
    if (dtype == COMAP_H5_STR_VLEN) return fail("comap_h5_write: use comap_h5_write_strings", -1);
    const std::string p = norm(path);
    if (comap_h5_delete(f, p.c_str())) return -2;
    Hid mt(mem_type(dtype, elsize));
    if (!mt.ok()) return fail("comap_h5_write: unsupported dtype", -1);
    Hid space;
    if (int rc = make_space(ndim, dims, space)) return rc;
    Hid lcpl(H5Pcreate(H5P_LINK_CREATE));
    H5Pset_create_intermediate_group(lcpl, 1);
    Hid d(H5Dcreate2(f->file, p.c_str(), mt, space, lcpl, H5P_DEFAULT, H5P_DEFAULT));
    if (!d.ok()) return fail("create dataset " + p);
    if (n_elements(ndim, dims) == 0) return 0;
    if (!buf) return fail("comap_h5_write: no buffer", -1);
    return H5Dwrite(d, mt, H5S_ALL, H5S_ALL, H5P_DEFAULT, buf) < 0 ? fail("write " + p) : 0;
}

int64_t comap_h5_read_strings(comap_h5 *f, const char *path, const char *attr, char *buf, int64_t cap)
{
    if (!valid(f) || !path) return fail("comap_h5_read_strings: bad arguments", -1);
    const std::string p = norm(path);
    if (attr) {
        Hid a(H5Aopen_by_name(f->file, p.c_str(), attr, H5P_DEFAULT, H5P_DEFAULT));
        if (!a.ok()) return fail("no attribute " + p + ":" + attr, -3);
        return read_vlen(a, true, buf, cap);
    }
    Hid d(H5Dopen2(f->file, p.c_str(), H5P_DEFAULT));
    if (!d.ok()) return fail("no dataset " + p, -3);
    return read_vlen(d, false, buf, cap);
}

int comap_h5_write_strings(comap_h5 *f, const char *path, const char *attr, int32_t ndim, const int64_t *dims,
                           const char *buf)
{
    if (!valid(f) || !path || (ndim > 0 && !dims)) return fail("comap_h5_write_strings: bad arguments", -1);
    const std::string p = norm(path);
    Hid mt(mem_type(COMAP_H5_STR_VLEN, 0)), space;
    if (int rc = make_space(ndim, dims, space)) return rc;
    const int64_t n = n_elements(ndim, dims);
    if (n > 0 && !buf) return fail("comap_h5_write_strings: no buffer", -1);
    std::vector<const char *> ptr = split_strings(buf, n);
    if (attr) {
        if (!path_exists(f->file, p)) return fail("no object " + p, -3);
        if (H5Aexists_by_name(f->file, p.c_str(), attr, H5P_DEFAULT) > 0 &&
            H5Adelete_by_name(f->file, p.c_str(), attr, H5P_DEFAULT) < 0)
            return fail("delete attribute " + p + ":" + attr);
        Hid a(H5Acreate_by_name(f->file, p.c_str(), attr, mt, space, H5P_DEFAULT, H5P_DEFAULT, H5P_DEFAULT));
        if (!a.ok()) return fail("create attribute " + p + ":" + attr);
        return H5Awrite(a, mt, ptr.data()) < 0 ? fail("write attribute " + p + ":" + attr) : 0;
    }
    if (comap_h5_delete(f, p.c_str())) return -2;
    Hid lcpl(H5Pcreate(H5P_LINK_CREATE));
    H5Pset_create_intermediate_group(lcpl, 1);
    Hid d(H5Dcreate2(f->file, p.c_str(), mt, space, lcpl, H5P_DEFAULT, H5P_DEFAULT));
    if (!d.ok()) return fail("create dataset " + p);
    if (n == 0) return 0;
    return H5Dwrite(d, mt, H5S_ALL, H5S_ALL, H5P_DEFAULT, ptr.data()) < 0 ? fail("write " + p) : 0;
}

int64_t comap_h5_attr_list(comap_h5 *f, const char *path, char *buf, int64_t cap)
{
    if (!valid(f) || !path) return fail("comap_h5_attr_list: bad arguments", -1);
    const std::string p = norm(path);
    Hid o(H5Oopen(f->file, p.c_str(), H5P_DEFAULT));
    if (!o.ok()) return fail("no object " + p, -3);
    std::string names;
    hsize_t idx = 0;
    if (H5Aiterate2(o, H5_INDEX_NAME, H5_ITER_INC, &idx, attr_cb, &names) < 0) return fail("H5Aiterate2");
    return put_text(names, buf, cap);
}

int comap_h5_attr_info(comap_h5 *f, const char *path, const char *name, int32_t *dtype, int32_t *ndim,
                       int64_t *dims, int64_t *elsize)
{
    if (!valid(f) || !path || !name || !dtype || !ndim || !dims || !elsize)
        return fail("comap_h5_attr_info: bad arguments", -1);
    Hid a(H5Aopen_by_name(f->file, norm(path).c_str(), name, H5P_DEFAULT, H5P_DEFAULT));
    if (!a.ok()) return fail(std::string("no attribute ") + path + ":" + name, -3);
    Hid t(H5Aget_type(a)), s(H5Aget_space(a));
    if (!t.ok() || !s.ok()) return fail("attribute type/space");
    *dtype = classify(t, elsize);
    return space_shape(s, ndim, dims);
}

int comap_h5_attr_read(comap_h5 *f, const char *path, const char *name, int32_t dtype, int64_t elsize, void *buf)
{
    if (!valid(f) || !path || !name || !buf) return fail("comap_h5_attr_read: bad arguments", -1);
    if (dtype == COMAP_H5_STR_VLEN) return fail("comap_h5_attr_read: use comap_h5_read_strings", -1);
    Hid a(H5Aopen_by_name(f->file, norm(path).c_str(), name, H5P_DEFAULT, H5P_DEFAULT));
    if (!a.ok()) return fail(std::string("no attribute ") + path + ":" + name, -3);
    Hid mt(mem_type(dtype, elsize));
    if (!mt.ok()) return fail("comap_h5_attr_read: unsupported dtype", -1);
    return H5Aread(a, mt, buf) < 0 ? fail(std::string("read attribute ") + path + ":" + name) : 0;
}

int comap_h5_attr_write(comap_h5 *f, const char *path, const char *name, int32_t dtype, int64_t elsize,
                        int32_t ndim, const int64_t *dims, const void *buf)
{
    if (!valid(f) || !path || !name || (ndim > 0 && !dims)) return fail("comap_h5_attr_write: bad arguments", -1);
    if (dtype == COMAP_H5_STR_VLEN) return fail("comap_h5_attr_write: use comap_h5_write_strings", -1);
    const std::string p = norm(path);
    if (!path_exists(f->file, p)) return fail("no object " + p, -3);
    Hid mt(mem_type(dtype, elsize)), space;
    if (!mt.ok()) return fail("comap_h5_attr_write: unsupported dtype", -1);
    if (int rc = make_space(ndim, dims, space)) return rc;
    if (H5Aexists_by_name(f->file, p.c_str(), name, H5P_DEFAULT) > 0 &&
        H5Adelete_by_name(f->file, p.c_str(), name, H5P_DEFAULT) < 0)
        return fail("delete attribute " + p + ":" + name);
    Hid a(H5Acreate_by_name(f->file, p.c_str(), name, mt, space, H5P_DEFAULT, H5P_DEFAULT, H5P_DEFAULT));
    if (!a.ok()) return fail("create attribute " + p + ":" + name);
    if (n_elements(ndim, dims) == 0) return 0;
    if (!buf) return fail("comap_h5_attr_write: no buffer", -1);
    return H5Awrite(a, mt, buf) < 0 ? fail("write attribute " + p + ":" + name) : 0;
}

}  // extern "C"
