// gguf.h -- GGUF v3 reader (mmap, zero-copy) and streaming writer.
//
// Replaces the ggml `gguf.h` parser the reference links against
// (src/gguf_loader.cpp:17-53, src/text_decoder.cpp:38-78, :270-335).  The
// reference mmaps the file (MAP_PRIVATE) and hands tensor pointers to ggml;
// here the mapped bytes are the staging source for one device arena upload.
#pragma once

#include <cstddef>
#include <cstdint>
#include <map>
#include <string>
#include <vector>

namespace qasr {

enum gguf_vtype : uint32_t {
    GV_U8 = 0, GV_I8 = 1, GV_U16 = 2, GV_I16 = 3, GV_U32 = 4, GV_I32 = 5, GV_F32 = 6,
    GV_BOOL = 7, GV_STR = 8, GV_ARR = 9, GV_U64 = 10, GV_I64 = 11, GV_F64 = 12,
};

// ggml tensor types used by the converter (scripts/convert_hf_to_gguf.py:254-311)
enum ggml_dtype : uint32_t { DT_F32 = 0, DT_F16 = 1, DT_Q8_0 = 8, DT_BF16 = 30 };

size_t ggml_row_bytes(uint32_t type, int64_t n);   // 0 for unsupported types

struct gguf_value {
    uint32_t type = 0;
    uint64_t u = 0;        // all integer / bool types
    int64_t i = 0;
    double f = 0;          // f32 / f64
    std::string s;
    uint32_t arr_type = 0;
    uint64_t arr_n = 0;
    size_t arr_off = 0;    // file offset of first array element
};

struct gguf_tensor {
    std::string name;
    uint32_t type = 0;
    std::vector<int64_t> ne;   // ggml order: ne[0] fastest
    uint64_t offset = 0;       // relative to data section
    size_t nbytes = 0;
    const uint8_t *data = nullptr;
    int64_t nelements() const {
        int64_t n = 1;
        for (auto v : ne) n *= v;
        return n;
    }
};

class GGUFFile {
public:
    ~GGUFFile();
    bool open(const std::string &path);
    void close();
    const std::string &error() const { return err_; }

    const gguf_value *find(const std::string &key) const;
    // reference semantics: gguf_get_val_u32 on a missing key -> default
    int64_t get_int(const std::string &key, int64_t def) const;
    double get_float(const std::string &key, double def) const;
    bool get_str_array(const std::string &key, std::vector<std::string> &out) const;

    const gguf_tensor *tensor(const std::string &name) const;
    const std::vector<gguf_tensor> &tensors() const { return tensors_; }
    uint32_t version() const { return version_; }
    size_t data_offset() const { return data_off_; }

private:
    bool parse();
    bool read_value(size_t &p, uint32_t type, gguf_value &v);
    bool skip_value(size_t &p, uint32_t type);
    bool rd(size_t &p, void *dst, size_t n);
    bool rd_str(size_t &p, std::string &s);

    int fd_ = -1;
    const uint8_t *base_ = nullptr;
    size_t size_ = 0;
    uint32_t version_ = 0;
    size_t data_off_ = 0;
    std::map<std::string, gguf_value> kv_;
    std::vector<gguf_tensor> tensors_;
    std::map<std::string, size_t> tindex_;
    std::string err_;
};

// Streaming writer: declare everything first, then write tensor bytes in
// declaration order through a callback (so 1.5 GB models never sit in RAM).
class GGUFWriter {
public:
    void add_u32(const std::string &k, uint32_t v);
    void add_f32(const std::string &k, float v);
    void add_str(const std::string &k, const std::string &v);
    void add_str_array(const std::string &k, const std::vector<std::string> &v);
    void add_tensor(const std::string &name, uint32_t type, const std::vector<int64_t> &ne);
    // fill(i, dst, nbytes) must write tensor i's bytes
    template <class F> bool write(const std::string &path, F fill);
    std::string error;

private:
    struct kvrec { std::string key; uint32_t type; std::vector<uint8_t> payload; };
    struct trec { std::string name; uint32_t type; std::vector<int64_t> ne; size_t nbytes; uint64_t off; };
    bool write_impl(const std::string &path, void *ctx, bool (*cb)(void *, size_t, uint8_t *, size_t));
    std::vector<kvrec> kvs_;
    std::vector<trec> ts_;
};

template <class F> bool GGUFWriter::write(const std::string &path, F fill) {
    auto cb = [](void *ctx, size_t i, uint8_t *dst, size_t n) -> bool { return (*(F *)ctx)(i, dst, n); };
    return write_impl(path, (void *)&fill, cb);
}

}  // namespace qasr
