// gguf.cpp -- GGUF v3 reader/writer (see gguf.h).
#include "gguf.h"

#include <cstdio>
#include <cstring>
#include <fcntl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

namespace qasr {

size_t ggml_row_bytes(uint32_t type, int64_t n) {
    switch (type) {
        case DT_F32: return (size_t)n * 4;
        case DT_F16: return (size_t)n * 2;
        case DT_BF16: return (size_t)n * 2;
        case DT_Q8_0: return (n % 32) ? 0 : (size_t)(n / 32) * 34;
        default: return 0;
    }
}

GGUFFile::~GGUFFile() { close(); }

void GGUFFile::close() {
    if (base_) munmap((void *)base_, size_);
    if (fd_ >= 0) ::close(fd_);
    base_ = nullptr;
    fd_ = -1;
    size_ = 0;
    kv_.clear();
    tensors_.clear();
    tindex_.clear();
}

bool GGUFFile::open(const std::string &path) {
    close();
    fd_ = ::open(path.c_str(), O_RDONLY);
    if (fd_ < 0) { err_ = "Failed to open GGUF file: " + path; return false; }
    struct stat st;
    if (fstat(fd_, &st) != 0) { err_ = "Failed to stat file: " + path; close(); return false; }
    size_ = (size_t)st.st_size;
    void *p = mmap(nullptr, size_, PROT_READ, MAP_PRIVATE, fd_, 0);
    if (p == MAP_FAILED) { err_ = "Failed to mmap file: " + path; base_ = nullptr; close(); return false; }
    base_ = (const uint8_t *)p;
    if (!parse()) { std::string e = err_; close(); err_ = e; return false; }
    return true;
}

bool GGUFFile::rd(size_t &p, void *dst, size_t n) {
    if (p + n > size_) { err_ = "GGUF: truncated file"; return false; }
    memcpy(dst, base_ + p, n);
    p += n;
    return true;
}

bool GGUFFile::rd_str(size_t &p, std::string &s) {
    uint64_t n;
    if (!rd(p, &n, 8)) return false;
    if (n > size_ || p + n > size_) { err_ = "GGUF: bad string length"; return false; }
    s.assign((const char *)base_ + p, n);
    p += n;
    return true;
}

static size_t scalar_size(uint32_t t) {
    switch (t) {
        case GV_U8: case GV_I8: case GV_BOOL: return 1;
        case GV_U16: case GV_I16: return 2;
        case GV_U32: case GV_I32: case GV_F32: return 4;
        case GV_U64: case GV_I64: case GV_F64: return 8;
        default: return 0;
    }
}

bool GGUFFile::skip_value(size_t &p, uint32_t type) {
    if (type == GV_STR) { std::string s; return rd_str(p, s); }
    size_t sz = scalar_size(type);
    if (!sz) { err_ = "GGUF: unknown value type"; return false; }
    if (p + sz > size_) { err_ = "GGUF: truncated value"; return false; }
    p += sz;
    return true;
}

bool GGUFFile::read_value(size_t &p, uint32_t type, gguf_value &v) {
    v.type = type;
    switch (type) {
        case GV_U8: { uint8_t x; if (!rd(p, &x, 1)) return false; v.u = x; v.i = x; return true; }
        case GV_I8: { int8_t x; if (!rd(p, &x, 1)) return false; v.i = x; v.u = (uint64_t)x; return true; }
        case GV_BOOL: { uint8_t x; if (!rd(p, &x, 1)) return false; v.u = x; v.i = x; return true; }
        case GV_U16: { uint16_t x; if (!rd(p, &x, 2)) return false; v.u = x; v.i = x; return true; }
        case GV_I16: { int16_t x; if (!rd(p, &x, 2)) return false; v.i = x; v.u = (uint64_t)x; return true; }
        case GV_U32: { uint32_t x; if (!rd(p, &x, 4)) return false; v.u = x; v.i = x; return true; }
        case GV_I32: { int32_t x; if (!rd(p, &x, 4)) return false; v.i = x; v.u = (uint64_t)x; return true; }
        case GV_U64: { uint64_t x; if (!rd(p, &x, 8)) return false; v.u = x; v.i = (int64_t)x; return true; }
        case GV_I64: { int64_t x; if (!rd(p, &x, 8)) return false; v.i = x; v.u = (uint64_t)x; return true; }
        case GV_F32: { float x; if (!rd(p, &x, 4)) return false; v.f = x; return true; }
        case GV_F64: { double x; if (!rd(p, &x, 8)) return false; v.f = x; return true; }
        case GV_STR: return rd_str(p, v.s);
        case GV_ARR: {
            if (!rd(p, &v.arr_type, 4) || !rd(p, &v.arr_n, 8)) return false;
            v.arr_off = p;
            if (v.arr_type == GV_STR) {
                for (uint64_t k = 0; k < v.arr_n; k++) if (!skip_value(p, GV_STR)) return false;
            } else if (v.arr_type == GV_ARR) {
                err_ = "GGUF: nested arrays unsupported";
                return false;
            } else {
                size_t sz = scalar_size(v.arr_type);
                if (!sz || v.arr_n > size_ || p + sz * v.arr_n > size_) { err_ = "GGUF: bad array"; return false; }
                p += sz * v.arr_n;
            }
            return true;
        }
        default: err_ = "GGUF: unknown value type " + std::to_string(type); return false;
    }
}

bool GGUFFile::parse() {
    size_t p = 0;
    uint32_t magic;
    if (!rd(p, &magic, 4)) return false;
    if (magic != 0x46554747u) { err_ = "GGUF: bad magic"; return false; }
    if (!rd(p, &version_, 4)) return false;
    if (version_ < 2 || version_ > 3) { err_ = "GGUF: unsupported version " + std::to_string(version_); return false; }
    uint64_t n_tensors, n_kv;
    if (!rd(p, &n_tensors, 8) || !rd(p, &n_kv, 8)) return false;
    if (n_tensors > (1u << 24) || n_kv > (1u << 24)) { err_ = "GGUF: implausible header counts"; return false; }
    for (uint64_t i = 0; i < n_kv; i++) {
        std::string key;
        uint32_t type;
        if (!rd_str(p, key) || !rd(p, &type, 4)) return false;
        gguf_value v;
        if (!read_value(p, type, v)) return false;
        kv_[key] = std::move(v);
    }
    tensors_.resize(n_tensors);
    for (uint64_t i = 0; i < n_tensors; i++) {
        gguf_tensor &t = tensors_[i];
        uint32_t nd;
        if (!rd_str(p, t.name) || !rd(p, &nd, 4)) return false;
        if (nd == 0 || nd > 4) { err_ = "GGUF: bad n_dims for " + t.name; return false; }
        t.ne.resize(nd);
        for (uint32_t d = 0; d < nd; d++) {
            uint64_t x;
            if (!rd(p, &x, 8)) return false;
            t.ne[d] = (int64_t)x;
        }
        if (!rd(p, &t.type, 4) || !rd(p, &t.offset, 8)) return false;
        size_t rb = ggml_row_bytes(t.type, t.ne[0]);
        int64_t rows = 1;
        for (uint32_t d = 1; d < nd; d++) rows *= t.ne[d];
        t.nbytes = rb * (size_t)rows;   // 0 => unsupported dtype (rejected at use)
        tindex_[t.name] = i;
    }
    uint64_t align = (uint64_t)get_int("general.alignment", 32);
    if (align == 0 || (align & (align - 1))) { err_ = "GGUF: bad alignment"; return false; }
    data_off_ = (p + align - 1) / align * align;
    for (auto &t : tensors_) {
        if (t.nbytes && data_off_ + t.offset + t.nbytes > size_) { err_ = "GGUF: tensor data out of file: " + t.name; return false; }
        t.data = base_ + data_off_ + t.offset;
    }
    return true;
}

const gguf_value *GGUFFile::find(const std::string &key) const {
    auto it = kv_.find(key);
    return it == kv_.end() ? nullptr : &it->second;
}

int64_t GGUFFile::get_int(const std::string &key, int64_t def) const {
    const gguf_value *v = find(key);
    if (!v) return def;
    if (v->type == GV_F32 || v->type == GV_F64) return (int64_t)v->f;
    return v->i;
}

double GGUFFile::get_float(const std::string &key, double def) const {
    const gguf_value *v = find(key);
    if (!v) return def;
    if (v->type == GV_F32 || v->type == GV_F64) return v->f;
    return (double)v->i;
}

bool GGUFFile::get_str_array(const std::string &key, std::vector<std::string> &out) const {
    const gguf_value *v = find(key);
    if (!v || v->type != GV_ARR || v->arr_type != GV_STR) return false;
    out.clear();
    out.reserve(v->arr_n);
    size_t p = v->arr_off;
    for (uint64_t k = 0; k < v->arr_n; k++) {
        uint64_t n;
        memcpy(&n, base_ + p, 8);
        p += 8;
        out.emplace_back((const char *)base_ + p, n);
        p += n;
    }
    return true;
}

const gguf_tensor *GGUFFile::tensor(const std::string &name) const {
    auto it = tindex_.find(name);
    return it == tindex_.end() ? nullptr : &tensors_[it->second];
}

// ---------------------------------------------------------------- writer
static void put(std::vector<uint8_t> &b, const void *p, size_t n) {
    const uint8_t *c = (const uint8_t *)p;
    b.insert(b.end(), c, c + n);
}
static void put_str(std::vector<uint8_t> &b, const std::string &s) {
    uint64_t n = s.size();
    put(b, &n, 8);
    put(b, s.data(), s.size());
}

void GGUFWriter::add_u32(const std::string &k, uint32_t v) {
    kvrec r{k, GV_U32, {}};
    put(r.payload, &v, 4);
    kvs_.push_back(std::move(r));
}
void GGUFWriter::add_f32(const std::string &k, float v) {
    kvrec r{k, GV_F32, {}};
    put(r.payload, &v, 4);
    kvs_.push_back(std::move(r));
}
void GGUFWriter::add_str(const std::string &k, const std::string &v) {
    kvrec r{k, GV_STR, {}};
    put_str(r.payload, v);
    kvs_.push_back(std::move(r));
}
void GGUFWriter::add_str_array(const std::string &k, const std::vector<std::string> &v) {
    kvrec r{k, GV_ARR, {}};
    uint32_t t = GV_STR;
    uint64_t n = v.size();
    put(r.payload, &t, 4);
    put(r.payload, &n, 8);
    for (auto &s : v) put_str(r.payload, s);
    kvs_.push_back(std::move(r));
}
void GGUFWriter::add_tensor(const std::string &name, uint32_t type, const std::vector<int64_t> &ne) {
    int64_t rows = 1;
    for (size_t d = 1; d < ne.size(); d++) rows *= ne[d];
    ts_.push_back({name, type, ne, ggml_row_bytes(type, ne[0]) * (size_t)rows, 0});
}

bool GGUFWriter::write_impl(const std::string &path, void *ctx, bool (*cb)(void *, size_t, uint8_t *, size_t)) {
    const uint64_t align = 32;
    std::vector<uint8_t> h;
    uint32_t magic = 0x46554747u, ver = 3;
    uint64_t nt = ts_.size(), nkv = kvs_.size();
    put(h, &magic, 4); put(h, &ver, 4); put(h, &nt, 8); put(h, &nkv, 8);
    for (auto &r : kvs_) {
        put_str(h, r.key);
        put(h, &r.type, 4);
        put(h, r.payload.data(), r.payload.size());
    }
    uint64_t off = 0;
    for (auto &t : ts_) {
        t.off = off;
        off += (t.nbytes + align - 1) / align * align;
        put_str(h, t.name);
        uint32_t nd = (uint32_t)t.ne.size();
        put(h, &nd, 4);
        for (auto v : t.ne) { uint64_t x = (uint64_t)v; put(h, &x, 8); }
        put(h, &t.type, 4);
        put(h, &t.off, 8);
    }
    while (h.size() % align) h.push_back(0);
    FILE *f = fopen(path.c_str(), "wb");
    if (!f) { error = "cannot create " + path; return false; }
    bool ok = fwrite(h.data(), 1, h.size(), f) == h.size();
    std::vector<uint8_t> buf;
    for (size_t i = 0; ok && i < ts_.size(); i++) {
        size_t padded = (ts_[i].nbytes + align - 1) / align * align;
        buf.assign(padded, 0);
        ok = cb(ctx, i, buf.data(), ts_[i].nbytes) && fwrite(buf.data(), 1, padded, f) == padded;
    }
    if (fclose(f) != 0) ok = false;
    if (!ok && error.empty()) error = "write failed: " + path;
    return ok;
}

}  // namespace qasr
