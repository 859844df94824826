// egs.cpp — Kaldi chain egs input for the MI355X core (include/kf_egs.h).
//
// Restates the reference's pure-Go egs path as a C-ABI library (libkaldi_fp16_egs.so):
//   internal/parser/parser.go   byte-scanning example reader (tags, I1V, CM/CM2/CM3/FM)
//   internal/parser/fst.go      OpenFst compact_acceptor / vector reader, deriv weights
//   internal/parser/matrix.go   matrix payloads + host decompression, SM/SV reader
//   internal/sparse/sparse.go   FST -> COO/CSR, merge, label dim, validation
//   internal/loader/*.go        file iterator + DataLoader.NextBatch
//   internal/batch/batch.go     feature / ivector merge
// The scanning state machine keeps the reference's exact byte semantics (it is what
// decides which bytes become matrices), including its tolerance of junk between tags.
// Deliberate differences, each an error path of the reference:
//   * a truncated FST, an absurd FST/string/matrix size or inconsistent compact offsets
//     give NULL / an error (the reference zero-fills short reads or panics);
//   * an FST whose header arc count disagrees with its arcs is rejected by the loader
//     (sparse.FstToCOO + COOToCSR index out of range / truncate there);
//   * shuffle uses a seeded Fisher-Yates (splitmix64) instead of Go's global rand.
// Matrices stay in stored form; the GPU expands them (csrc/egs.hip) straight into the
// fp16 network input, so the host never materialises the fp32 batch on the hot path.
#include <glob.h>
#include <hip/hip_runtime_api.h>
#include <zlib.h>

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdarg>
#include <cstdio>
#include <cstring>
#include <memory>
#include <string>
#include <vector>

#include "../../include/kf_egs.h"
#include "../../include/kf_ops.h"

namespace {

thread_local std::string g_err;

void set_err(const char *fmt, ...) {
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof(buf), fmt, ap);
    va_end(ap);
    g_err = buf;
}

// ------------------------------------------------------------------ byte source
// bufio.Reader semantics the parser relies on: ReadByte (0 + false at EOF), a one-byte
// UnreadByte valid right after a successful ReadByte, and io.ReadFull.
class ByteSrc {
  public:
    static std::unique_ptr<ByteSrc> from_file(FILE *f) {
        auto s = std::unique_ptr<ByteSrc>(new ByteSrc);
        s->f_ = f;
        s->buf_.resize(1 + kChunk);
        return s;
    }
    static std::unique_ptr<ByteSrc> from_gz(gzFile g) {
        auto s = std::unique_ptr<ByteSrc>(new ByteSrc);
        s->gz_ = g;
        s->buf_.resize(1 + kChunk);
        return s;
    }
    static std::unique_ptr<ByteSrc> from_mem(const uint8_t *p, size_t n) {
        auto s = std::unique_ptr<ByteSrc>(new ByteSrc);
        s->mem_ = p;
        s->len_ = n;
        return s;
    }
    ~ByteSrc() {
        if (f_) fclose(f_);
        if (gz_) gzclose(gz_);
    }
    bool read_byte(uint8_t &b) {
        if (pos_ >= len_ && !fill()) {
            b = 0;
            can_unread_ = false;
            return false;
        }
        b = data()[pos_++];
        consumed_++;
        can_unread_ = true;
        return true;
    }
    void unread() {
        if (can_unread_ && pos_ > 0) {
            pos_--;
            consumed_--;
        }
        can_unread_ = false;
    }
    // io.ReadFull: bytes actually read (short only at EOF); the rest of dst untouched
    size_t read_full(void *dst, size_t n) {
        uint8_t *d = static_cast<uint8_t *>(dst);
        size_t got = 0;
        can_unread_ = false;
        while (got < n) {
            if (pos_ >= len_ && !fill()) break;
            const size_t k = std::min(n - got, len_ - pos_);
            memcpy(d + got, data() + pos_, k);
            pos_ += k;
            got += k;
        }
        consumed_ += got;
        return got;
    }
    size_t consumed() const { return consumed_; }

  private:
    static constexpr size_t kChunk = 1 << 16;
    ByteSrc() = default;
    const uint8_t *data() const { return mem_ ? mem_ : buf_.data(); }
    bool fill() {
        if (mem_ || (!f_ && !gz_)) return false;
        // keep the last byte so an UnreadByte right after a refill still works
        size_t keep = 0;
        if (len_ > 0) {
            buf_[0] = buf_[len_ - 1];
            keep = 1;
        }
        long n = 0;
        if (f_)
            n = (long)fread(buf_.data() + keep, 1, kChunk, f_);
        else
            n = gzread(gz_, buf_.data() + keep, (unsigned)kChunk);
        if (n <= 0) {
            if (keep) {
                pos_ = len_ = 1;
            }
            return false;
        }
        pos_ = keep;
        len_ = keep + (size_t)n;
        return true;
    }
    FILE *f_ = nullptr;
    gzFile gz_ = nullptr;
    const uint8_t *mem_ = nullptr;
    std::vector<uint8_t> buf_;
    size_t pos_ = 0, len_ = 0, consumed_ = 0;
    bool can_unread_ = false;
};

// scalar reads ignore short reads like the reference's helpers (zero-filled)
int32_t rd_i32(ByteSrc &s) {
    uint8_t b[4] = {0, 0, 0, 0};
    s.read_full(b, 4);
    int32_t v;
    memcpy(&v, b, 4);
    return v;
}
float rd_f32(ByteSrc &s) {
    uint8_t b[4] = {0, 0, 0, 0};
    s.read_full(b, 4);
    float v;
    memcpy(&v, b, 4);
    return v;
}
// strict variants for the FST reader (truncation -> failure)
bool rd_exact(ByteSrc &s, void *dst, size_t n) { return s.read_full(dst, n) == n; }

bool is_letter(uint8_t b) { return (b >= 'a' && b <= 'z') || (b >= 'A' && b <= 'Z'); }
bool is_digit(uint8_t b) { return b >= '0' && b <= '9'; }

// readBasicIntValue (parser.go:434-445): space, size byte, 1 -> unsigned byte, 4 -> int32
int32_t rd_basic_int(ByteSrc &s) {
    uint8_t b;
    s.read_byte(b);
    uint8_t size;
    s.read_byte(size);
    if (size == 1) {
        uint8_t v;
        s.read_byte(v);
        return (int32_t)v;
    }
    if (size == 4) return rd_i32(s);
    return 0;
}
// readBasicInt32 / readBasicFloat32 (matrix.go:229-249): size must be 4
int32_t rd_basic_i32_strict(ByteSrc &s) {
    uint8_t b;
    s.read_byte(b);
    uint8_t size;
    s.read_byte(size);
    if (size != 4) return -1;
    return rd_i32(s);
}
float rd_basic_f32_strict(ByteSrc &s) {
    uint8_t b;
    s.read_byte(b);
    uint8_t size;
    s.read_byte(size);
    if (size != 4) return 0.f;
    return rd_f32(s);
}

// ------------------------------------------------------------------ owned objects
struct FstOwned {
    int64_t start = 0, num_states = 0, num_arcs = 0;
    uint64_t properties = 0;
    std::vector<int32_t> arc_off, label, next;
    std::vector<float> weight, final_w;
    KfEgsFst view() const {
        KfEgsFst v;
        v.start = start;
        v.num_states = num_states;
        v.num_arcs = num_arcs;
        v.properties = properties;
        v.arc_off = arc_off.data();
        v.label = label.data();
        v.weight = weight.data();
        v.next_state = next.data();
        v.final_weight = final_w.data();
        return v;
    }
};

struct IoOwned {
    std::string name;
    std::vector<int32_t> idx;  // [n][3]
    int format = KF_MAT_NONE, rows = 0, cols = 0;
    float mn = 0, rg = 0;
    std::vector<uint8_t> payload;
};

struct ExOwned {
    std::string key;
    int num_inputs = 0, num_outputs = 0;
    std::vector<IoOwned> io;
    std::string sup_name;
    std::vector<int32_t> sup_idx;
    float weight = 0;
    int nseq = 0, fps = 0, label_dim = 0, e2e = 0;
    bool has_fst = false;
    FstOwned fst;
    bool has_dw = false;
    std::vector<float> dw;

    std::vector<KfEgsIo> io_view;
    KfEgsExample view;
    void build_view() {
        io_view.resize(io.size());
        for (size_t i = 0; i < io.size(); i++) {
            KfEgsIo &v = io_view[i];
            const IoOwned &o = io[i];
            v.name = o.name.c_str();
            v.num_indexes = (int)(o.idx.size() / 3);
            v.indexes = o.idx.data();
            v.format = o.format;
            v.rows = o.rows;
            v.cols = o.cols;
            v.min_value = o.mn;
            v.range = o.rg;
            v.payload = o.payload.data();
            v.payload_bytes = o.payload.size();
        }
        memset(&view, 0, sizeof(view));
        view.key = key.c_str();
        view.num_inputs = num_inputs;
        view.num_outputs = num_outputs;
        view.num_io = (int)io.size();
        view.io = io_view.data();
        view.sup_name = sup_name.c_str();
        view.sup_num_indexes = (int)(sup_idx.size() / 3);
        view.sup_indexes = sup_idx.data();
        view.weight = weight;
        view.num_sequences = nseq;
        view.frames_per_seq = fps;
        view.label_dim = label_dim;
        view.end2end = e2e;
        view.has_fst = has_fst ? 1 : 0;
        if (has_fst) view.fst = fst.view();
        view.num_deriv_weights = (int)dw.size();
        view.deriv_weights = dw.data();
    }
};

void copy_from_view(const KfEgsExample &v, ExOwned &o) {
    o.key = v.key ? v.key : "";
    o.num_inputs = v.num_inputs;
    o.num_outputs = v.num_outputs;
    o.io.resize(v.num_io > 0 ? v.num_io : 0);
    for (int i = 0; i < v.num_io; i++) {
        const KfEgsIo &s = v.io[i];
        IoOwned &d = o.io[i];
        d.name = s.name ? s.name : "";
        d.idx.assign(s.indexes, s.indexes + 3 * (size_t)std::max(0, s.num_indexes));
        d.format = s.format;
        d.rows = s.rows;
        d.cols = s.cols;
        d.mn = s.min_value;
        d.rg = s.range;
        d.payload.assign(s.payload, s.payload + s.payload_bytes);
    }
    o.sup_name = v.sup_name ? v.sup_name : "";
    o.sup_idx.assign(v.sup_indexes, v.sup_indexes + 3 * (size_t)std::max(0, v.sup_num_indexes));
    o.weight = v.weight;
    o.nseq = v.num_sequences;
    o.fps = v.frames_per_seq;
    o.label_dim = v.label_dim;
    o.e2e = v.end2end;
    o.has_fst = v.has_fst != 0;
    if (o.has_fst) {
        const KfEgsFst &f = v.fst;
        FstOwned &g = o.fst;
        g.start = f.start;
        g.num_states = f.num_states;
        g.num_arcs = f.num_arcs;
        g.properties = f.properties;
        g.arc_off.assign(f.arc_off, f.arc_off + f.num_states + 1);
        const size_t na = (size_t)g.arc_off[f.num_states];
        g.label.assign(f.label, f.label + na);
        g.weight.assign(f.weight, f.weight + na);
        g.next.assign(f.next_state, f.next_state + na);
        g.final_w.assign(f.final_weight, f.final_weight + f.num_states);
    }
    o.has_dw = v.num_deriv_weights > 0;
    o.dw.assign(v.deriv_weights, v.deriv_weights + std::max(0, v.num_deriv_weights));
    o.build_view();
}

// ------------------------------------------------------------------ FST (fst.go)
constexpr int32_t kFstMagic = 0x7eb2fdd6;
constexpr int64_t kMaxFstStates = 1LL << 26;
constexpr uint32_t kMaxFstString = 1u << 12;

bool rd_fst_string(ByteSrc &s, std::string &out) {  // readString (fst.go:301-309)
    uint32_t n;
    if (!rd_exact(s, &n, 4) || n > kMaxFstString) return false;
    out.resize(n);
    return n == 0 || rd_exact(s, &out[0], n);
}

// ReadFst (fst.go:18-172). false on a bad magic, type, or truncation.
bool read_fst(ByteSrc &s, FstOwned &f) {
    int32_t magic;
    if (!rd_exact(s, &magic, 4) || magic != kFstMagic) {
        set_err("FST: bad magic");
        return false;
    }
    std::string fst_type, arc_type;
    if (!rd_fst_string(s, fst_type) || !rd_fst_string(s, arc_type)) {
        set_err("FST: truncated header strings");
        return false;
    }
    if (arc_type != "standard") {
        set_err("FST: arc type '%s' (want standard)", arc_type.c_str());
        return false;
    }
    const bool compact = fst_type == "compact_acceptor";
    if (!compact && fst_type != "vector") {
        set_err("FST: type '%s' (want compact_acceptor or vector)", fst_type.c_str());
        return false;
    }
    struct {
        int32_t version, flags;
        uint64_t properties;
        int64_t start, num_states, num_arcs;
    } h;
    if (!rd_exact(s, &h.version, 4) || !rd_exact(s, &h.flags, 4) || !rd_exact(s, &h.properties, 8) ||
        !rd_exact(s, &h.start, 8) || !rd_exact(s, &h.num_states, 8) || !rd_exact(s, &h.num_arcs, 8)) {
        set_err("FST: truncated header");
        return false;
    }
    if (h.num_states < 0 || h.num_states > kMaxFstStates) {
        set_err("FST: %lld states", (long long)h.num_states);
        return false;
    }
    const int64_t S = h.num_states;
    f.start = h.start;
    f.num_states = S;
    f.properties = h.properties;
    f.arc_off.assign(S + 1, 0);
    f.final_w.assign(S, INFINITY);
    f.label.clear();
    f.weight.clear();
    f.next.clear();
    if (compact) {
        std::vector<uint32_t> off(S + 1);
        if (!rd_exact(s, off.data(), 4 * (S + 1))) {
            set_err("FST: truncated state offsets");
            return false;
        }
        const uint32_t nc = off[S];
        for (int64_t i = 0; i < S; i++)
            if (off[i] > off[i + 1]) {
                set_err("FST: state offsets not monotonic at %lld", (long long)i);
                return false;
            }
        if (nc > (uint32_t)(kMaxFstStates * 16)) {
            set_err("FST: %u compacts", nc);
            return false;
        }
        std::vector<int32_t> el(3 * (size_t)nc);
        if (nc && !rd_exact(s, el.data(), 12 * (size_t)nc)) {
            set_err("FST: truncated compacts");
            return false;
        }
        for (int64_t st = 0; st < S; st++) {
            for (uint32_t i = off[st]; i < off[st + 1]; i++) {
                float w;
                memcpy(&w, &el[3 * i + 1], 4);
                if (el[3 * i + 2] == -1) {
                    f.final_w[st] = w;  // kNoStateId: final weight, the last one wins
                } else {
                    f.label.push_back(el[3 * i]);
                    f.weight.push_back(w);
                    f.next.push_back(el[3 * i + 2]);
                }
            }
            f.arc_off[st + 1] = (int32_t)f.label.size();
        }
        f.num_arcs = h.num_arcs;  // header value, as the reference keeps it
    } else {
        for (int64_t st = 0; st < S; st++) {
            float fw;
            int64_t narcs;
            if (!rd_exact(s, &fw, 4) || !rd_exact(s, &narcs, 8) || narcs < 0 || narcs > kMaxFstStates) {
                set_err("FST: truncated or bad vector state %lld", (long long)st);
                return false;
            }
            f.final_w[st] = fw;
            for (int64_t a = 0; a < narcs; a++) {
                int32_t rec[4];
                if (!rd_exact(s, rec, 16)) {
                    set_err("FST: truncated vector arcs");
                    return false;
                }
                float w;
                memcpy(&w, &rec[2], 4);
                f.label.push_back(rec[0]);  // ilabel (olabel == ilabel for an acceptor)
                f.weight.push_back(w);
                f.next.push_back(rec[3]);
            }
            f.arc_off[st + 1] = (int32_t)f.label.size();
        }
        f.num_arcs = (int64_t)f.label.size();  // the vector header holds 0
    }
    return true;
}

// readDerivWeights (fst.go:232-267)
void read_deriv_weights(ByteSrc &s, const std::string &tag, ExOwned &ex) {
    uint8_t b, f1, f2;
    s.read_byte(b);
    s.read_byte(f1);
    s.read_byte(f2);
    ex.has_dw = true;
    ex.dw.clear();
    if (f1 != 'F' || f2 != 'V') return;
    s.read_byte(b);
    if (tag == "DW") {
        const int32_t n = rd_i32(s);
        for (int32_t i = 0; i < n; i++) {
            uint8_t v;
            s.read_byte(v);
            ex.dw.push_back((float)v / 255.0f);
        }
    } else {
        s.read_byte(b);  // size byte
        const int32_t n = rd_i32(s);
        for (int32_t i = 0; i < n; i++) ex.dw.push_back(rd_f32(s));
    }
}

// ------------------------------------------------------------------ matrices (matrix.go)
// CM / CM2 / CM3 / FM payload readers. NULL-equivalent (false) on bad dims or short
// data, exactly where the reference's read*/Read* return nil.
bool read_matrix(ByteSrc &s, int kind, IoOwned &m) {
    int64_t bytes;
    if (kind == KF_MAT_FM) {
        uint8_t size;
        s.read_byte(size);
        if (size != 4) return false;
        m.mn = m.rg = 0;
        m.rows = rd_i32(s);
        m.cols = rd_i32(s);
        if (m.rows <= 0 || m.cols <= 0) return false;
        bytes = 4LL * m.rows * m.cols;
        if (bytes > (1LL << 31)) return false;  // unbounded in the reference
    } else {
        m.mn = rd_f32(s);
        m.rg = rd_f32(s);
        m.rows = rd_i32(s);
        m.cols = rd_i32(s);
        if (m.rows <= 0 || m.cols <= 0 || m.rows > 100000 || m.cols > 10000) return false;
        const int64_t rc = (int64_t)m.rows * m.cols;
        bytes = kind == KF_MAT_CM ? 8LL * m.cols + rc : kind == KF_MAT_CM2 ? 2 * rc : rc;
    }
    m.format = kind;
    m.payload.resize((size_t)bytes);
    return s.read_full(m.payload.data(), (size_t)bytes) == (size_t)bytes;
}

float u16_to_float(float mn, float rg, uint16_t v) {  // matrix.go:11-14
    const float inv65535 = 1.52590218966964e-05f;
    volatile float a = rg * inv65535;  // one rounding per Go float32 op
    volatile float b = a * (float)v;
    return mn + b;
}

float char_to_float(float p0, float p25, float p75, float p100, uint8_t v) {  // matrix.go:17-26
    if (v <= 64) {
        volatile float d = p25 - p0;
        volatile float m = d * (float)v;
        volatile float q = m * (1.0f / 64.0f);
        return p0 + q;
    }
    if (v <= 192) {
        volatile float d = p75 - p25;
        volatile float m = d * (float)(uint8_t)(v - 64);
        volatile float q = m * (1.0f / 128.0f);
        return p25 + q;
    }
    volatile float d = p100 - p75;
    volatile float m = d * (float)(uint8_t)(v - 192);
    return (float)((double)p75 + (double)m / 63.0);
}

int decompress(const KfEgsIo &m, float *out) {
    const int R = m.rows, Cc = m.cols;
    const size_t rc = (size_t)R * Cc;
    const uint8_t *p = m.payload;
    switch (m.format) {
    case KF_MAT_CM: {
        if (m.payload_bytes < 8 * (size_t)Cc + rc) return -1;
        for (int c = 0; c < Cc; c++) {
            uint16_t hv[4];
            memcpy(hv, p + 8 * (size_t)c, 8);
            const float p0 = u16_to_float(m.min_value, m.range, hv[0]);
            const float p25 = u16_to_float(m.min_value, m.range, hv[1]);
            const float p75 = u16_to_float(m.min_value, m.range, hv[2]);
            const float p100 = u16_to_float(m.min_value, m.range, hv[3]);
            const uint8_t *col = p + 8 * (size_t)Cc + (size_t)c * R;
            for (int r = 0; r < R; r++) out[(size_t)r * Cc + c] = char_to_float(p0, p25, p75, p100, col[r]);
        }
        return 0;
    }
    case KF_MAT_CM2: {
        if (m.payload_bytes < 2 * rc) return -1;
        volatile float inc = m.range / 65535.0f;
        for (size_t i = 0; i < rc; i++) {
            uint16_t v;
            memcpy(&v, p + 2 * i, 2);
            volatile float t = (float)v * inc;
            out[i] = m.min_value + t;
        }
        return 0;
    }
    case KF_MAT_CM3: {
        if (m.payload_bytes < rc) return -1;
        volatile float inc = m.range / 255.0f;
        for (size_t i = 0; i < rc; i++) {
            volatile float t = (float)p[i] * inc;
            out[i] = m.min_value + t;
        }
        return 0;
    }
    case KF_MAT_FM:
        if (m.payload_bytes < 4 * rc) return -1;
        memcpy(out, p, 4 * rc);
        return 0;
    }
    return -1;
}

// ------------------------------------------------------------------ example parser
// tryReadTag (parser.go:387-413)
bool try_read_tag(ByteSrc &s, std::string &tag) {
    tag.clear();
    for (;;) {
        uint8_t b;
        if (!s.read_byte(b)) return false;
        if (b == '>') break;
        if (b == ' ') {
            s.unread();
            break;
        }
        if (!is_letter(b) && !is_digit(b) && b != '/' && b != '_') return false;
        tag.push_back((char)b);
        if (tag.size() > 30) return false;
    }
    return tag.size() >= 2;
}

// readName (parser.go:415-432)
std::string read_name(ByteSrc &s) {
    uint8_t b;
    const bool ok = s.read_byte(b);
    if (ok && b != ' ') s.unread();
    std::string name;
    for (;;) {
        const bool got = s.read_byte(b);
        if (!got || b == ' ' || b == '<') {
            if (got && b == '<') s.unread();
            break;
        }
        name.push_back((char)b);
    }
    return name;
}

// readIndexVector (parser.go:484-548); returns indexes decoded, -1 on count <= 0
int read_index_vector(ByteSrc &s, int count, std::vector<int32_t> &out, bool &eof) {
    eof = false;
    out.clear();
    if (count <= 0) return -1;
    out.reserve(3 * (size_t)count);
    for (int i = 0; i < count; i++) {
        uint8_t b;
        if (!s.read_byte(b)) {
            eof = true;
            return i;
        }
        const int8_t c = (int8_t)b;
        int32_t n, t, x;
        if (c == 127) {  // long form: three WriteBasicType ints
            n = rd_basic_int(s);
            t = rd_basic_int(s);
            x = rd_basic_int(s);
        } else if (i == 0) {  // delta (the out-of-range deltas decode the same way)
            n = 0;
            t = c;
            x = 0;
        } else {
            n = out[3 * (i - 1)];
            t = out[3 * (i - 1) + 1] + c;
            x = out[3 * (i - 1) + 2];
        }
        out.push_back(n);
        out.push_back(t);
        out.push_back(x);
    }
    return count;
}

// findExampleStart (parser.go:128-160)
bool find_example_start(ByteSrc &s, std::string &key) {
    std::string kb;
    bool in_key = false;
    for (;;) {
        uint8_t b;
        if (!s.read_byte(b)) return false;
        if (!in_key) {
            if (is_letter(b)) {
                in_key = true;
                kb.assign(1, (char)b);
            }
            continue;
        }
        if (is_letter(b) || is_digit(b) || b == '-' || b == '_' || b == '.') {
            kb.push_back((char)b);
            continue;
        }
        if (b == ' ' && kb.size() >= 3) {
            uint8_t b2, b3;
            s.read_byte(b2);
            if (b2 == 0) {
                s.read_byte(b3);
                if (b3 == 'B') {
                    key = kb;
                    return true;
                }
            }
        }
        in_key = false;
        kb.clear();
    }
}

// parseExample (parser.go:163-302). 0 = complete example, -1 = error (g_err set).
int parse_example(ByteSrc &s, ExOwned &ex) {
    std::string cur_name;
    std::vector<int32_t> cur_idx;
    for (;;) {
        uint8_t b;
        if (!s.read_byte(b)) {
            set_err("unexpected EOF");
            return -1;
        }
        if ((b == 'C' || b == 'F') && !cur_name.empty()) {
            uint8_t b2;
            if (!s.read_byte(b2)) continue;
            int kind = KF_MAT_NONE;
            if (b == 'C' && b2 == 'M') {
                uint8_t b3;
                if (!s.read_byte(b3)) continue;
                if (b3 == '2') {
                    s.read_byte(b3);
                    kind = KF_MAT_CM2;
                } else if (b3 == '3') {
                    s.read_byte(b3);
                    kind = KF_MAT_CM3;
                } else if (b3 == ' ') {
                    kind = KF_MAT_CM;
                } else {
                    s.unread();
                    continue;
                }
            } else if (b == 'F' && b2 == 'M') {
                uint8_t b3;
                s.read_byte(b3);
                if (b3 == ' ') {
                    kind = KF_MAT_FM;
                } else {
                    s.unread();
                    continue;
                }
            } else {
                s.unread();
                continue;
            }
            IoOwned m;
            if (read_matrix(s, kind, m)) {
                m.name = cur_name;
                m.idx = cur_idx;
                ex.io.push_back(std::move(m));
                cur_name.clear();
            }
            continue;
        }
        if (b != '<') continue;
        std::string tag;
        if (!try_read_tag(s, tag)) continue;
        if (tag == "NumInputs") {
            ex.num_inputs = rd_basic_int(s);
        } else if (tag == "NumOutputs") {
            ex.num_outputs = rd_basic_int(s);
        } else if (tag == "NnetIo") {
            cur_name = read_name(s);
        } else if (tag == "I1V") {
            const int count = rd_basic_int(s);
            std::vector<int32_t> idx;
            bool eof;
            const int got = read_index_vector(s, count, idx, eof);
            if (got < 0 || eof) {
                set_err("I1V read error (name=%s): %s", cur_name.c_str(),
                        got < 0 ? "invalid index vector count" : "EOF inside index vector");
                return -1;
            }
            if (!cur_name.empty())
                cur_idx = std::move(idx);
            else if (!ex.sup_name.empty())
                ex.sup_idx = std::move(idx);
        } else if (tag == "/NnetIo") {
            cur_name.clear();
        } else if (tag == "NnetChainSup") {
            ex.sup_name = read_name(s);
        } else if (tag == "Weight") {
            uint8_t t;
            s.read_byte(t);
            s.read_byte(t);
            ex.weight = rd_f32(s);
        } else if (tag == "NumSequences") {
            ex.nseq = rd_basic_int(s);
        } else if (tag == "FramesPerSeq") {
            ex.fps = rd_basic_int(s);
        } else if (tag == "LabelDim") {
            ex.label_dim = rd_basic_int(s);
        } else if (tag == "End2End") {
            uint8_t t, e;
            s.read_byte(t);
            s.read_byte(e);
            ex.e2e = e == 'T';
            if (!ex.e2e) {
                if (!read_fst(s, ex.fst)) {
                    const std::string why = g_err;
                    set_err("failed to read FST for example (%s)", why.c_str());
                    return -1;
                }
                ex.has_fst = true;
            }
        } else if (tag == "DW" || tag == "DW2") {
            read_deriv_weights(s, tag, ex);
        } else if (tag == "/Nnet3ChainEg") {
            return 0;
        }
    }
}

}  // namespace

// ====================================================================== reader API
// a parsed FST handed to the caller: the C view plus the arrays it points into
struct FstPack : KfEgsFst {
    FstOwned o;
};

struct KfEgsReader {
    std::unique_ptr<ByteSrc> src;
    ExOwned cur;
};

extern "C" {

const char *kf_egs_last_error(void) { return g_err.empty() ? nullptr : g_err.c_str(); }
void kf_egs_clear_error(void) { g_err.clear(); }

int kf_egs_detect_format(const char *path) {
    FILE *f = path ? fopen(path, "rb") : nullptr;
    if (!f) {
        set_err("cannot open %s", path ? path : "(null)");
        return -1;
    }
    uint8_t buf[256];
    const size_t n = fread(buf, 1, sizeof(buf), f);
    fclose(f);
    if (n < 10) {
        set_err("file too small or unreadable (%zu bytes)", n);
        return -1;
    }
    for (size_t i = 0; i + 1 < n; i++)
        if (buf[i] == 0 && buf[i + 1] == 'B') return 0;
    for (size_t i = 0; i < n; i++)
        if (buf[i] == '\n') {
            set_err("text ark format detected (no binary \\0B marker found), only binary ark files supported");
            return -1;
        }
    set_err("unknown format (no binary \\0B marker found in first %zu bytes)", n);
    return -1;
}

KfEgsReader *kf_egs_open(const char *path) {
    if (!path) {
        set_err("kf_egs_open: null path");
        return nullptr;
    }
    const size_t L = strlen(path);
    const bool gz = L >= 3 && strcmp(path + L - 3, ".gz") == 0;
    if (!gz && kf_egs_detect_format(path) != 0) {
        const std::string why = g_err;
        set_err("format check failed for %s: %s", path, why.c_str());
        return nullptr;
    }
    auto r = std::unique_ptr<KfEgsReader>(new KfEgsReader);
    if (gz) {
        // gzip.NewReader validates the header up front: check the magic the same way
        FILE *f = fopen(path, "rb");
        if (!f) {
            set_err("cannot open %s", path);
            return nullptr;
        }
        uint8_t m[2] = {0, 0};
        const size_t n = fread(m, 1, 2, f);
        fclose(f);
        if (n != 2 || m[0] != 0x1f || m[1] != 0x8b) {
            set_err("gzip reader failed for %s: invalid header", path);
            return nullptr;
        }
        gzFile g = gzopen(path, "rb");
        if (!g) {
            set_err("gzip reader failed for %s", path);
            return nullptr;
        }
        gzbuffer(g, 1 << 17);
        r->src = ByteSrc::from_gz(g);
    } else {
        FILE *f = fopen(path, "rb");
        if (!f) {
            set_err("cannot open %s", path);
            return nullptr;
        }
        r->src = ByteSrc::from_file(f);
    }
    return r.release();
}

int kf_egs_next(KfEgsReader *r, const KfEgsExample **out) {
    if (!r || !out) {
        set_err("kf_egs_next: null argument");
        return -1;
    }
    *out = nullptr;
    std::string key;
    if (!find_example_start(*r->src, key)) return 0;
    r->cur = ExOwned();
    if (parse_example(*r->src, r->cur) != 0) return -1;
    r->cur.key = key;
    r->cur.build_view();
    *out = &r->cur.view;
    return 1;
}

void kf_egs_close(KfEgsReader *r) { delete r; }

int kf_egs_example_valid(const KfEgsExample *ex) {  // parser.go:463-474
    if (!ex || ex->num_inputs != 2 || ex->num_outputs != 1 || ex->num_io != 2) return 0;
    const KfEgsIo &a = ex->io[0], &b = ex->io[1];
    if (strcmp(a.name, "input") != 0 || a.cols != 40) return 0;
    if (strcmp(b.name, "ivector") != 0 || b.rows != 1 || b.cols != 100) return 0;
    return 1;
}

int kf_egs_example_usable(const KfEgsExample *ex) {  // parser.go:477-479
    return kf_egs_example_valid(ex) && ex->weight > 0 && ex->label_dim == 3080;
}

int kf_egs_io_to_float(const KfEgsIo *io, float *out) {
    if (!io || !out || io->rows <= 0 || io->cols <= 0) {
        set_err("kf_egs_io_to_float: bad arguments");
        return -1;
    }
    if (decompress(*io, out) != 0) {
        set_err("kf_egs_io_to_float: format %d payload %zu bytes too short for %dx%d", io->format,
                io->payload_bytes, io->rows, io->cols);
        return -1;
    }
    return 0;
}

int kf_egs_parse_index_vector(const uint8_t *buf, size_t len, int count, int32_t *out, int *n_read,
                              size_t *used) {
    auto s = ByteSrc::from_mem(buf, buf ? len : 0);
    std::vector<int32_t> idx;
    bool eof;
    const int got = read_index_vector(*s, count, idx, eof);
    if (used) *used = s->consumed();
    if (n_read) *n_read = got < 0 ? 0 : got;
    if (got > 0 && out) memcpy(out, idx.data(), idx.size() * 4);
    if (got < 0) {
        set_err("invalid index vector count: %d", count);
        return -1;
    }
    if (eof) {
        set_err("EOF after %d/%d indexes", got, count);
        return -1;
    }
    return 0;
}

KfEgsFst *kf_egs_parse_fst(const uint8_t *buf, size_t len, size_t *used) {
    auto s = ByteSrc::from_mem(buf, buf ? len : 0);
    auto f = std::unique_ptr<FstOwned>(new FstOwned);
    const bool ok = read_fst(*s, *f);
    if (used) *used = s->consumed();
    if (!ok) return nullptr;
    FstPack *p = new FstPack;
    p->o = std::move(*f);
    static_cast<KfEgsFst &>(*p) = p->o.view();
    return p;
}

void kf_egs_fst_free(KfEgsFst *f) { delete static_cast<FstPack *>(f); }

int kf_egs_parse_sparse_matrix(const uint8_t *buf, size_t len, int32_t *row_dim, int32_t *row_off,
                               int32_t *pair_index, float *pair_value, int *num_pairs, size_t *used) {
    // ReadSparseMatrix (matrix.go:172-226)
    auto s = ByteSrc::from_mem(buf, buf ? len : 0);
    const int32_t nrows = rd_basic_i32_strict(*s);
    if (nrows <= 0 || nrows > 10000000) {
        if (used) *used = s->consumed();
        set_err("SM: invalid num_rows %d", nrows);
        return -1;
    }
    std::vector<int32_t> dims, offs(1, 0), idx;
    std::vector<float> val;
    for (int i = 0; i < nrows; i++) {
        uint8_t a, b;
        s->read_byte(a);
        s->read_byte(b);
        if (a != 'S' || b != 'V') {
            if (used) *used = s->consumed();
            set_err("SM: row %d: expected SV token", i);
            return -1;
        }
        const int32_t dim = rd_basic_i32_strict(*s);
        const int32_t ne = rd_basic_i32_strict(*s);
        if (dim < 0 || ne < 0 || ne > dim) {
            if (used) *used = s->consumed();
            set_err("SM: row %d: dim %d elems %d", i, dim, ne);
            return -1;
        }
        for (int k = 0; k < ne; k++) {
            idx.push_back(rd_basic_i32_strict(*s));
            val.push_back(rd_basic_f32_strict(*s));
        }
        dims.push_back(dim);
        offs.push_back((int32_t)idx.size());
    }
    if (used) *used = s->consumed();
    if (num_pairs) *num_pairs = (int)idx.size();
    if (row_dim) memcpy(row_dim, dims.data(), dims.size() * 4);
    if (row_off) memcpy(row_off, offs.data(), offs.size() * 4);
    if (pair_index && !idx.empty()) memcpy(pair_index, idx.data(), idx.size() * 4);
    if (pair_value && !val.empty()) memcpy(pair_value, val.data(), val.size() * 4);
    return nrows;
}

int kf_egs_fst_to_csr(const KfEgsFst *f, int32_t *row_ptr, int32_t *col, int32_t *label, float *logw,
                      int32_t *final_state, float *final_logw, int *num_finals) {
    // FstToCSR (sparse.go:54-102)
    if (!f) {
        set_err("nil FST");
        return -1;
    }
    if (f->num_states <= 0) {
        set_err("FST has no states");
        return -1;
    }
    const int64_t S = f->num_states;
    const int32_t A = f->arc_off[S];
    if ((int64_t)A != f->num_arcs) {
        set_err("arc count mismatch: counted %d, expected %lld", A, (long long)f->num_arcs);
        return -1;
    }
    int nf = 0;
    for (int64_t i = 0; i < S; i++) {
        if (row_ptr) row_ptr[i] = f->arc_off[i];
        for (int32_t a = f->arc_off[i]; a < f->arc_off[i + 1]; a++) {
            if (col) col[a] = f->next_state[a];
            if (label) label[a] = f->label[a];
            if (logw) logw[a] = -f->weight[a];
        }
        if (!(std::isinf(f->final_weight[i]) && f->final_weight[i] > 0)) {  // not +Inf
            if (final_state) final_state[nf] = (int32_t)i;
            if (final_logw) final_logw[nf] = -f->final_weight[i];
            nf++;
        }
    }
    if (row_ptr) row_ptr[S] = A;
    if (num_finals) *num_finals = nf;
    return 0;
}

}  // extern "C"

// ====================================================================== batch
struct KfEgsBatch {
    std::vector<ExOwned> ex;
    int total_frames = 0, feat_dim = 0, ivec_dim = 0, label_dim = 0, num_sequences = 0;
    float weight = 0;
    std::vector<int32_t> frame_off, nframes, fps, state_offsets;
    // merged CSR
    std::vector<int32_t> row_ptr, col, label, final_state;
    std::vector<float> logw, final_logw;
    // per-example layout
    std::vector<int32_t> state_off, arc_off, final_off, per_row_ptr, per_col, per_final_state;
    size_t upload_bytes = 0;
};

namespace {

// validateExample (dataloader.go:229-249)
bool validate_example(const ExOwned &e, std::string &why) {
    if (e.io.empty()) return why = "no inputs", false;
    if (e.io[0].name != "input") return why = "first input is '" + e.io[0].name + "', expected 'input'", false;
    if (e.io[0].rows <= 0 || e.io[0].cols <= 0) return why = "invalid input matrix", false;
    if (!e.has_fst) return why = "supervision FST is nil", false;
    if (!(e.weight > 0)) return why = "zero or negative weight", false;
    return true;
}

// batch.NewBatch (batch.go:43-123) sizes + mergeFSTs (dataloader.go:252-277)
bool assemble(KfEgsBatch &b) {
    const int B = (int)b.ex.size();
    for (ExOwned &e : b.ex) e.build_view();  // the vector may have moved the strings
    if (B == 0) {
        set_err("empty examples list");
        return false;
    }
    b.frame_off.assign(B, 0);
    b.nframes.assign(B, 0);
    b.fps.assign(B, 0);
    int total = 0, fd = 0, iv = 0;
    for (int i = 0; i < B; i++) {
        const ExOwned &e = b.ex[i];
        if (e.io.empty()) {
            set_err("example %d (%s): no inputs", i, e.key.c_str());
            return false;
        }
        const IoOwned &in = e.io[0];
        if (in.name != "input") {
            set_err("example %d (%s): first input is '%s', expected 'input'", i, e.key.c_str(), in.name.c_str());
            return false;
        }
        b.frame_off[i] = total;
        b.nframes[i] = in.rows;
        total += in.rows;
        if (fd == 0)
            fd = in.cols;
        else if (in.cols != fd) {
            set_err("example %d (%s): feat_dim=%d, expected %d", i, e.key.c_str(), in.cols, fd);
            return false;
        }
        if (e.io.size() >= 2 && e.io[1].name == "ivector" && iv == 0) iv = e.io[1].cols;
        b.fps[i] = e.fps;
    }
    b.total_frames = total;
    b.feat_dim = fd;
    b.ivec_dim = iv;
    b.num_sequences = b.ex[0].nseq;
    b.weight = b.ex[0].weight;

    // FST -> COO per example (sparse.go:105-142), merged with state offsets (:217-261),
    // COOToCSR (:173-212) — the arcs are already grouped by source state, so the stable
    // sort is the identity.
    b.state_off.assign(B + 1, 0);
    b.arc_off.assign(B + 1, 0);
    b.final_off.assign(B + 1, 0);
    b.state_offsets.assign(B, 0);
    for (int i = 0; i < B; i++) {
        const FstOwned &f = b.ex[i].fst;
        if (f.num_states <= 0) {
            set_err("FST merge failed: example %d (%s): FST has no states", i, b.ex[i].key.c_str());
            return false;
        }
        if (f.num_arcs != (int64_t)f.label.size()) {
            set_err("FST merge failed: example %d (%s): header arcs %lld != %zu arcs", i,
                    b.ex[i].key.c_str(), (long long)f.num_arcs, f.label.size());
            return false;
        }
        b.state_offsets[i] = b.state_off[i];
        b.state_off[i + 1] = b.state_off[i] + (int32_t)f.num_states;
        b.arc_off[i + 1] = b.arc_off[i] + (int32_t)f.label.size();
    }
    const int S = b.state_off[B], A = b.arc_off[B];
    b.row_ptr.assign(S + 1, 0);
    b.col.resize(A);
    b.label.resize(A);
    b.logw.resize(A);
    b.per_row_ptr.resize(S + B);
    b.per_col.resize(A);
    b.final_state.clear();
    b.final_logw.clear();
    b.per_final_state.clear();
    int maxl = 0;
    for (int i = 0; i < B; i++) {
        const FstOwned &f = b.ex[i].fst;
        const int so = b.state_off[i], ao = b.arc_off[i];
        for (int64_t st = 0; st <= f.num_states; st++) {
            b.per_row_ptr[so + i + st] = f.arc_off[st];
            if (st < f.num_states) b.row_ptr[so + st] = ao + f.arc_off[st];
        }
        for (size_t a = 0; a < f.label.size(); a++) {
            b.col[ao + a] = f.next[a] + so;
            b.per_col[ao + a] = f.next[a];
            b.label[ao + a] = f.label[a];
            b.logw[ao + a] = -f.weight[a];
            maxl = std::max(maxl, f.label[a]);
        }
        for (int64_t st = 0; st < f.num_states; st++)
            if (!(std::isinf(f.final_w[st]) && f.final_w[st] > 0)) {
                b.final_state.push_back(so + (int32_t)st);
                b.per_final_state.push_back((int32_t)st);
                b.final_logw.push_back(-f.final_w[st]);
            }
        b.final_off[i + 1] = (int32_t)b.final_state.size();
    }
    b.row_ptr[S] = A;
    b.label_dim = maxl + 1;
    for (int a = 0; a < A; a++)  // CSR.Validate (sparse.go:286-318)
        if (b.col[a] < 0 || b.col[a] >= S) {
            set_err("merged CSR validation failed: ColIdx[%d] = %d out of range [0, %d)", a, b.col[a], S);
            return false;
        }
    return true;
}

int cm_format(int kind) {
    switch (kind) {
    case KF_MAT_CM: return KF_CM_ONEBYTE_COLHDR;
    case KF_MAT_CM2: return KF_CM_TWOBYTE;
    case KF_MAT_CM3: return KF_CM_ONEBYTE;
    case KF_MAT_FM: return KF_CM_FLOAT;
    }
    return 0;
}

// appends one matrix to the packed upload (4-byte aligned payloads)
void pack(std::vector<uint8_t> &blob, std::vector<KfCmDesc> &desc, const IoOwned &m, int rows, int out_row) {
    while (blob.size() % 4) blob.push_back(0);
    KfCmDesc d;
    d.format = cm_format(m.format);
    d.rows = rows;
    d.cols = m.cols;
    d.out_row = out_row;
    d.min_value = m.mn;
    d.range = m.rg;
    d.payload_off = (long long)blob.size();
    desc.push_back(d);
    blob.insert(blob.end(), m.payload.begin(), m.payload.end());
}

}  // namespace

extern "C" {

KfEgsBatch *kf_egs_batch_from_examples(const KfEgsExample *const *ex, int n) {
    if (!ex || n <= 0) {
        set_err("empty examples list");
        return nullptr;
    }
    auto b = std::unique_ptr<KfEgsBatch>(new KfEgsBatch);
    b->ex.resize(n);
    for (int i = 0; i < n; i++) {
        if (!ex[i]) {
            set_err("example %d is NULL", i);
            return nullptr;
        }
        copy_from_view(*ex[i], b->ex[i]);
    }
    if (!assemble(*b)) return nullptr;
    return b.release();
}

void kf_egs_batch_free(KfEgsBatch *b) { delete b; }

int kf_egs_batch_info(const KfEgsBatch *b, KfEgsBatchInfo *o) {
    if (!b || !o) {
        set_err("kf_egs_batch_info: null argument");
        return -1;
    }
    o->batch_size = (int)b->ex.size();
    o->total_frames = b->total_frames;
    o->feat_dim = b->feat_dim;
    o->ivector_dim = b->ivec_dim;
    o->label_dim = b->label_dim;
    o->num_sequences = b->num_sequences;
    o->weight = b->weight;
    o->frame_offsets = b->frame_off.data();
    o->num_frames = b->nframes.data();
    o->frames_per_seq = b->fps.data();
    o->state_offsets = b->state_offsets.data();
    o->num_states = (int)b->row_ptr.size() - 1;
    o->num_arcs = (int)b->col.size();
    o->num_finals = (int)b->final_state.size();
    o->row_ptr = b->row_ptr.data();
    o->col = b->col.data();
    o->label = b->label.data();
    o->logw = b->logw.data();
    o->final_state = b->final_state.data();
    o->final_logw = b->final_logw.data();
    o->state_off = b->state_off.data();
    o->arc_off = b->arc_off.data();
    o->final_off = b->final_off.data();
    o->per_row_ptr = b->per_row_ptr.data();
    o->per_col = b->per_col.data();
    o->per_final_state = b->per_final_state.data();
    return 0;
}

const char *kf_egs_batch_key(const KfEgsBatch *b, int i) {
    if (!b || i < 0 || i >= (int)b->ex.size()) return nullptr;
    return b->ex[i].key.c_str();
}

int kf_egs_batch_features_host(const KfEgsBatch *b, float *out) {
    if (!b || !out) {
        set_err("kf_egs_batch_features_host: null argument");
        return -1;
    }
    for (size_t i = 0; i < b->ex.size(); i++) {
        const ExOwned &e = b->ex[i];
        if (decompress(e.io_view[0], out + (size_t)b->frame_off[i] * b->feat_dim) != 0) {
            set_err("example %zu: bad feature payload", i);
            return -1;
        }
    }
    return 0;
}

int kf_egs_batch_ivectors_host(const KfEgsBatch *b, float *out) {
    if (!b || !out) {
        set_err("kf_egs_batch_ivectors_host: null argument");
        return -1;
    }
    const int D = b->ivec_dim;
    if (D == 0) return 0;
    memset(out, 0, sizeof(float) * b->ex.size() * D);
    std::vector<float> tmp;
    for (size_t i = 0; i < b->ex.size(); i++) {
        const ExOwned &e = b->ex[i];
        if (e.io.size() < 2 || e.io[1].name != "ivector") continue;
        const IoOwned &m = e.io[1];
        tmp.resize((size_t)m.rows * m.cols);
        if (decompress(e.io_view[1], tmp.data()) != 0) {
            set_err("example %zu: bad ivector payload", i);
            return -1;
        }
        const size_t n = std::min(tmp.size(), (size_t)D);  // Go copy() semantics
        memcpy(out + i * D, tmp.data(), n * 4);
    }
    return 0;
}

int kf_egs_batch_features(KfEgsBatch *b, void *dev_out, int ldo, void *dev_ivec) {
    if (!b || !dev_out || ldo < b->feat_dim) {
        set_err("kf_egs_batch_features: bad arguments (ldo %d, feat_dim %d)", ldo, b ? b->feat_dim : -1);
        return -1;
    }
    std::vector<uint8_t> blob;
    std::vector<KfCmDesc> desc;
    int max_rows = 1;
    for (size_t i = 0; i < b->ex.size(); i++) {
        const IoOwned &m = b->ex[i].io[0];
        pack(blob, desc, m, m.rows, b->frame_off[i]);
        max_rows = std::max(max_rows, m.rows);
    }
    size_t up = blob.size() + desc.size() * sizeof(KfCmDesc);
    if (kf_cm_expand_host(desc.data(), (int)desc.size(), max_rows, b->feat_dim, blob.data(), blob.size(),
                          dev_out, ldo) != 0) {
        set_err("features: %s", kf_last_error() ? kf_last_error() : "kf_cm_expand_host failed");
        return -1;
    }
    if (dev_ivec && b->ivec_dim > 0) {
        const int D = b->ivec_dim;
        blob.clear();
        desc.clear();
        for (size_t i = 0; i < b->ex.size(); i++) {
            const ExOwned &e = b->ex[i];
            if (e.io.size() < 2 || e.io[1].name != "ivector") continue;
            if (e.io[1].cols != D) {
                set_err("ivectors: example %zu has %d columns, the batch %d (use kf_egs_batch_ivectors_host)",
                        i, e.io[1].cols, D);
                return -1;
            }
            pack(blob, desc, e.io[1], 1, (int)i);  // first row, as copy() into Row(i) takes
        }
        if (desc.size() < b->ex.size() &&
            hipMemsetAsync(dev_ivec, 0, b->ex.size() * (size_t)D * 2, (hipStream_t)kf_get_stream()) != hipSuccess) {
            set_err("ivectors: memset failed");
            return -1;
        }
        up += blob.size() + desc.size() * sizeof(KfCmDesc);
        if (!desc.empty() && kf_cm_expand_host(desc.data(), (int)desc.size(), 1, D, blob.data(), blob.size(),
                                               dev_ivec, D) != 0) {
            set_err("ivectors: %s", kf_last_error() ? kf_last_error() : "kf_cm_expand_host failed");
            return -1;
        }
    }
    b->upload_bytes = up;
    return 0;
}

size_t kf_egs_batch_upload_bytes(const KfEgsBatch *b) { return b ? b->upload_bytes : 0; }

}  // extern "C"

// ====================================================================== loader
struct KfEgsLoader {
    std::vector<std::string> paths;
    size_t current = 0;
    KfEgsReader *reader = nullptr;
    int batch_size = 0;
    bool shuffle = false, drop_last = false;
    unsigned long long rng = 0;
    int batches = 0, examples = 0;
    double seconds = 0;
    ~KfEgsLoader() { kf_egs_close(reader); }

    uint64_t next_rand() {  // splitmix64
        uint64_t z = (rng += 0x9e3779b97f4a7c15ULL);
        z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ULL;
        z = (z ^ (z >> 27)) * 0x94d049bb133111ebULL;
        return z ^ (z >> 31);
    }
    void do_shuffle() {
        for (size_t i = paths.size(); i > 1; i--) std::swap(paths[i - 1], paths[next_rand() % i]);
    }
    // EgsIterator.Next (loader.go:69-103): 1 example, 0 exhausted, -1 error in a file
    int next(const KfEgsExample **ex) {
        for (;;) {
            if (!reader) {
                if (current >= paths.size()) return 0;
                reader = kf_egs_open(paths[current].c_str());
                if (!reader) {
                    current++;
                    continue;
                }
            }
            const int r = kf_egs_next(reader, ex);
            if (r < 0) {
                kf_egs_close(reader);
                reader = nullptr;
                current++;
                return -1;
            }
            if (r == 0) {
                kf_egs_close(reader);
                reader = nullptr;
                current++;
                continue;
            }
            return 1;
        }
    }
};

extern "C" {

KfEgsLoader *kf_egs_loader_create(const char *pattern, int batch_size, int shuffle, unsigned long long seed,
                                  int drop_last) {
    if (batch_size <= 0) {
        set_err("batch size must be > 0, got %d", batch_size);
        return nullptr;
    }
    if (!pattern) {
        set_err("null pattern");
        return nullptr;
    }
    auto l = std::unique_ptr<KfEgsLoader>(new KfEgsLoader);
    if (strchr(pattern, '\n')) {  // NewEgsIteratorFromPaths (loader.go:46-64)
        const char *p = pattern;
        while (*p) {
            const char *e = strchr(p, '\n');
            const size_t n = e ? (size_t)(e - p) : strlen(p);
            if (n) l->paths.emplace_back(p, n);
            p += n + (e ? 1 : 0);
        }
        if (l->paths.empty()) {
            set_err("failed to create iterator: empty paths list");
            return nullptr;
        }
    } else {  // NewEgsIterator (loader.go:22-43): filepath.Glob, sorted
        glob_t g;
        memset(&g, 0, sizeof(g));
        const int rc = glob(pattern, 0, nullptr, &g);
        if (rc == 0)
            for (size_t i = 0; i < g.gl_pathc; i++) l->paths.emplace_back(g.gl_pathv[i]);
        globfree(&g);
        if (l->paths.empty()) {
            set_err("failed to create iterator: no files match pattern: %s", pattern);
            return nullptr;
        }
    }
    l->batch_size = batch_size;
    l->shuffle = shuffle != 0;
    l->drop_last = drop_last != 0;
    l->rng = seed;
    if (l->shuffle) l->do_shuffle();
    return l.release();
}

int kf_egs_loader_next(KfEgsLoader *l, KfEgsBatch **out) {
    if (!l || !out) {
        set_err("kf_egs_loader_next: null argument");
        return -1;
    }
    *out = nullptr;
    const auto t0 = std::chrono::steady_clock::now();
    auto b = std::unique_ptr<KfEgsBatch>(new KfEgsBatch);
    while ((int)b->ex.size() < l->batch_size) {
        const KfEgsExample *v = nullptr;
        const int r = l->next(&v);
        if (r < 0) continue;  // skip errors (dataloader.go:106-112)
        if (r == 0) break;
        const KfEgsReader *rd = l->reader;
        std::string why;
        if (!validate_example(rd->cur, why)) continue;
        b->ex.push_back(rd->cur);  // deep copy; assemble() rebuilds the views
        l->examples++;
    }
    if (b->ex.empty()) return 0;
    if ((int)b->ex.size() < l->batch_size && l->drop_last) return 0;
    if (!assemble(*b)) {
        const std::string why = g_err;
        set_err("batch assembly failed: %s", why.c_str());
        return -1;
    }
    l->batches++;
    l->seconds += std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    *out = b.release();
    return 1;
}

void kf_egs_loader_reset(KfEgsLoader *l) {  // dataloader.go:187-193 + loader.go:107-119
    if (!l) return;
    kf_egs_close(l->reader);
    l->reader = nullptr;
    l->current = 0;
    if (l->shuffle) l->do_shuffle();
    l->batches = l->examples = 0;
    l->seconds = 0;
}

void kf_egs_loader_stats(const KfEgsLoader *l, int *batches, int *examples, double *seconds) {
    if (!l) return;
    if (batches) *batches = l->batches;
    if (examples) *examples = l->examples;
    if (seconds) *seconds = l->seconds;
}

int kf_egs_loader_num_files(const KfEgsLoader *l) { return l ? (int)l->paths.size() : 0; }

void kf_egs_loader_free(KfEgsLoader *l) { delete l; }

}  // extern "C"
