// nnet3_import.cpp — Kaldi nnet3 text model import (include/kf_model.h).
//
// ParseNnet3Text (internal/nnet/weight_loader.go:608-727) is restated line for line:
// the same substring tests, the same order of tag checks, the same treatment of a
// matrix opened on a tag line ("[" with no "]": the data starts on the next line and
// anything after "[" on the tag line is ignored), and Go's strconv rules for numbers
// (a token that does not parse, or overflows float32, is skipped).
// nnet_load_kaldi restates LoadWeights / NewNetworkFromKaldi (:65-437, :750-1104)
// on top of the public nnet_* ABI, so the import never touches network internals.
#include <cerrno>
#include <cmath>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <string>
#include <vector>

#include "../../include/kf_model.h"
#include "../../include/kf_nnet.h"

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

struct Comp {
    std::string name, type;
    std::vector<float> linear, bias, mean, var;
    int rows = 0, cols = 0;
    double count = 0;
    float eps = 0, rms = 0;
    int nfi = 0, nfo = 0, hin = 0, hout = 0, heads = 0, kdim = 0, vdim = 0;
    float kscale = 0, lr = 0, maxc = 0, l2 = 0;
};

// strings.Fields
std::vector<std::string> fields(const std::string &s, size_t from = 0) {
    std::vector<std::string> out;
    size_t i = from;
    while (i < s.size()) {
        while (i < s.size() && isspace((unsigned char)s[i])) ++i;
        size_t j = i;
        while (j < s.size() && !isspace((unsigned char)s[j])) ++j;
        if (j > i) out.emplace_back(s, i, j - i);
        i = j;
    }
    return out;
}

bool is_inf_literal(const std::string &t) {
    std::string u;
    for (char c : t) u.push_back((char)tolower((unsigned char)c));
    if (!u.empty() && (u[0] == '+' || u[0] == '-')) u.erase(0, 1);
    return u == "inf" || u == "infinity";
}

// strconv.ParseFloat(tok, 32): ok = syntactically valid; an overflow returns +-Inf with
// an error (the callers that ignore the error keep the Inf, parseFloatLine skips it)
bool parse_f32(const std::string &tok, float &v, bool &range_err) {
    range_err = false;
    if (tok.empty()) return false;
    std::string low;
    for (char c : tok) low.push_back((char)tolower((unsigned char)c));
    if (low.find("nan(") != std::string::npos || low.find('_') != std::string::npos) return false;
    errno = 0;
    char *end = nullptr;
    const float f = strtof(tok.c_str(), &end);
    if (!end || *end != '\0') return false;
    if (std::isinf(f) && !is_inf_literal(tok)) range_err = true;
    v = f;
    return true;
}

bool parse_f64(const std::string &tok, double &v, bool &range_err) {
    range_err = false;
    if (tok.empty()) return false;
    std::string low;
    for (char c : tok) low.push_back((char)tolower((unsigned char)c));
    if (low.find("nan(") != std::string::npos || low.find('_') != std::string::npos) return false;
    char *end = nullptr;
    const double f = strtod(tok.c_str(), &end);
    if (!end || *end != '\0') return false;
    if (std::isinf(f) && !is_inf_literal(tok)) range_err = true;
    v = f;
    return true;
}

// parseFloatLine (:1166-1177)
std::vector<float> parse_float_line(const std::string &line) {
    std::vector<float> out;
    for (const auto &f : fields(line)) {
        float v;
        bool re;
        if (parse_f32(f, v, re) && !re) out.push_back(v);
    }
    return out;
}

// first whitespace field after `tag`, unless absent or another tag
bool tag_field(const std::string &line, const char *tag, std::string &tok) {
    const size_t idx = line.find(tag);
    if (idx == std::string::npos) return false;
    auto fs = fields(line, idx + strlen(tag));
    if (fs.empty() || fs[0][0] == '<') return false;
    tok = fs[0];
    return true;
}

float tag_f32(const std::string &line, const char *tag) {  // parseFloat32Tag (:1179-1190)
    std::string t;
    float v;
    bool re;
    if (!tag_field(line, tag, t) || !parse_f32(t, v, re)) return 0.f;
    return v;  // ParseFloat's +-Inf on overflow is kept
}

double tag_f64(const std::string &line, const char *tag) {  // parseFloat64 (:1192-1203)
    std::string t;
    double v;
    bool re;
    if (!tag_field(line, tag, t) || !parse_f64(t, v, re)) return 0.0;
    return v;
}

int tag_int(const std::string &line, const char *tag) {  // parseIntTag / strconv.Atoi (:1205-1216)
    std::string t;
    if (!tag_field(line, tag, t)) return 0;
    size_t i = 0;
    if (t[0] == '+' || t[0] == '-') i = 1;
    if (i >= t.size()) return 0;
    for (size_t k = i; k < t.size(); ++k)
        if (!isdigit((unsigned char)t[k])) return 0;
    errno = 0;
    const long long v = strtoll(t.c_str(), nullptr, 10);
    if (errno == ERANGE || v > 2147483647LL || v < -2147483648LL) return 0;  // Atoi range error -> 0
    return (int)v;
}

// parseComponentHeader (:1118-1145)
Comp parse_header(const std::string &line) {
    Comp c;
    const size_t idx = line.find("<ComponentName>");
    if (idx == std::string::npos) return c;
    auto parts = fields(line, idx + strlen("<ComponentName>"));
    if (parts.size() < 2) return c;
    c.name = parts[0];
    std::string t = parts[1];  // strings.Trim(parts[1], "<>")
    size_t a = 0, b = t.size();
    while (a < b && (t[a] == '<' || t[a] == '>')) ++a;
    while (b > a && (t[b - 1] == '<' || t[b - 1] == '>')) --b;
    c.type = t.substr(a, b - a);
    c.lr = tag_f32(line, "<LearningRate>");
    c.maxc = tag_f32(line, "<MaxChange>");
    c.l2 = tag_f32(line, "<L2Regularize>");
    c.eps = tag_f32(line, "<Epsilon>");
    c.rms = tag_f32(line, "<TargetRms>");
    c.count = tag_f64(line, "<Count>");
    c.nfi = tag_int(line, "<NumFiltersIn>");
    c.nfo = tag_int(line, "<NumFiltersOut>");
    c.hin = tag_int(line, "<HeightIn>");
    c.hout = tag_int(line, "<HeightOut>");
    c.heads = tag_int(line, "<NumHeads>");
    c.kdim = tag_int(line, "<KeyDim>");
    c.vdim = tag_int(line, "<ValueDim>");
    c.kscale = tag_f32(line, "<KeyScale>");
    return c;
}

// finishMatrix (:1147-1164)
void finish(Comp &c, const std::string &tag, std::vector<float> &data, int rows) {
    if (data.empty()) return;
    const int cols = rows > 0 ? (int)(data.size() / rows) : 0;
    if (tag == "<LinearParams>" || tag == "<Params>") {
        c.linear = std::move(data);
        c.rows = rows;
        c.cols = cols;
    } else if (tag == "<BiasParams>") {
        c.bias = std::move(data);
    } else if (tag == "<StatsMean>") {
        c.mean = std::move(data);
    } else if (tag == "<StatsVar>") {
        c.var = std::move(data);
    }
    data.clear();
}

}  // namespace

struct KfNnet3Model {
    std::vector<Comp> comps;           // first-appearance order
    std::map<std::string, int> index;  // name -> slot (the last definition wins)
    void put(Comp &&c) {
        auto it = index.find(c.name);
        if (it != index.end()) {
            comps[it->second] = std::move(c);
        } else {
            index[c.name] = (int)comps.size();
            comps.push_back(std::move(c));
        }
    }
    const Comp *get(const std::string &n) const {
        auto it = index.find(n);
        return it == index.end() ? nullptr : &comps[it->second];
    }
};

extern "C" {

const char *kf_nnet3_last_error(void) { return g_err.empty() ? nullptr : g_err.c_str(); }

KfNnet3Model *kf_nnet3_parse_text(const char *text, size_t len) {
    if (!text) {
        set_err("kf_nnet3_parse_text: null text");
        return nullptr;
    }
    auto *m = new KfNnet3Model;
    static const char *kTags[] = {"<LinearParams>", "<Params>", "<BiasParams>", "<StatsMean>", "<StatsVar>"};
    bool have = false, in_matrix = false;
    Comp cur;
    std::vector<float> buf;
    int rows = 0;
    std::string mtag;
    size_t pos = 0;
    while (pos < len) {  // bufio.Scanner lines: split at '\n', drop one trailing '\r'
        size_t e = pos;
        while (e < len && text[e] != '\n') ++e;
        std::string line(text + pos, e - pos);
        if (!line.empty() && line.back() == '\r') line.pop_back();
        pos = e + 1;

        if (line.find("<ComponentName>") != std::string::npos) {
            if (have && in_matrix) finish(cur, mtag, buf, rows);
            if (have) m->put(std::move(cur));
            cur = parse_header(line);
            have = true;
            buf.clear();
            rows = 0;
            in_matrix = false;
            mtag.clear();
        }
        if (!have) continue;
        if (line.find("<Count>") != std::string::npos) cur.count = tag_f64(line, "<Count>");
        if (line.find("<Epsilon>") != std::string::npos && cur.eps == 0) cur.eps = tag_f32(line, "<Epsilon>");
        if (line.find("<TargetRms>") != std::string::npos && cur.rms == 0) cur.rms = tag_f32(line, "<TargetRms>");

        for (const char *tag : kTags) {
            if (line.find(tag) == std::string::npos) continue;
            if (in_matrix) finish(cur, mtag, buf, rows);
            mtag = tag;
            buf.clear();
            rows = 0;
            in_matrix = true;
            const size_t b = line.find('[');
            if (b != std::string::npos) {
                std::string after = line.substr(b + 1);
                const size_t c = after.find(']');
                if (c != std::string::npos) {
                    after = after.substr(0, c);
                    auto vals = parse_float_line(after);
                    if (!vals.empty()) {
                        buf = std::move(vals);
                        rows = 1;
                    }
                    finish(cur, mtag, buf, rows);
                    in_matrix = false;
                }
            }
            break;
        }
        if (in_matrix && line.find('<') == std::string::npos) {
            size_t a = 0, z = line.size();  // strings.TrimSpace
            while (a < z && isspace((unsigned char)line[a])) ++a;
            while (z > a && isspace((unsigned char)line[z - 1])) --z;
            std::string t = line.substr(a, z - a);
            if (t.empty()) continue;
            const size_t cb = t.find(']');
            const bool close = cb != std::string::npos;
            if (close) t.erase(cb, 1);
            auto vals = parse_float_line(t);
            if (!vals.empty()) {
                buf.insert(buf.end(), vals.begin(), vals.end());
                rows++;
            }
            if (close) {
                finish(cur, mtag, buf, rows);
                in_matrix = false;
            }
        }
    }
    if (have) {
        if (in_matrix) finish(cur, mtag, buf, rows);
        m->put(std::move(cur));
    }
    return m;
}

KfNnet3Model *kf_nnet3_read_text_file(const char *path) {
    FILE *f = path ? fopen(path, "rb") : nullptr;
    if (!f) {
        set_err("cannot open %s", path ? path : "(null)");
        return nullptr;
    }
    std::string s;
    char chunk[1 << 16];
    size_t n;
    while ((n = fread(chunk, 1, sizeof(chunk), f)) > 0) s.append(chunk, n);
    fclose(f);
    return kf_nnet3_parse_text(s.data(), s.size());
}

KfNnet3Model *kf_nnet3_export(const char *mdl_path) {
    if (!mdl_path) {
        set_err("kf_nnet3_export: null path");
        return nullptr;
    }
    std::string q = "'";
    for (const char *p = mdl_path; *p; ++p) {
        if (*p == '\'') q += "'\\''";
        else q.push_back(*p);
    }
    q += "'";
    const std::string cmd = "nnet3-copy --binary=false " + q + " - 2>/dev/null";
    FILE *p = popen(cmd.c_str(), "r");
    if (!p) {
        set_err("nnet3-copy failed: cannot start");
        return nullptr;
    }
    std::string s;
    char chunk[1 << 16];
    size_t n;
    while ((n = fread(chunk, 1, sizeof(chunk), p)) > 0) s.append(chunk, n);
    const int rc = pclose(p);
    if (rc != 0) {
        set_err("nnet3-copy failed: exit status %d (is Kaldi's nnet3-copy on PATH?)", rc);
        return nullptr;
    }
    return kf_nnet3_parse_text(s.data(), s.size());
}

void kf_nnet3_free(KfNnet3Model *m) { delete m; }

int kf_nnet3_num_components(const KfNnet3Model *m) { return m ? (int)m->comps.size() : 0; }

int kf_nnet3_find(const KfNnet3Model *m, const char *name) {
    if (!m || !name) return -1;
    auto it = m->index.find(name);
    return it == m->index.end() ? -1 : it->second;
}

int kf_nnet3_component(const KfNnet3Model *m, int idx, KfNnet3Component *o) {
    if (!m || !o || idx < 0 || idx >= (int)m->comps.size()) {
        set_err("kf_nnet3_component: bad index %d", idx);
        return -1;
    }
    const Comp &c = m->comps[idx];
    o->name = c.name.c_str();
    o->type = c.type.c_str();
    o->linear = c.linear.empty() ? nullptr : c.linear.data();
    o->linear_rows = c.linear.empty() ? 0 : c.rows;
    o->linear_cols = c.linear.empty() ? 0 : c.cols;
    o->bias = c.bias.empty() ? nullptr : c.bias.data();
    o->bias_dim = (int)c.bias.size();
    o->stats_mean = c.mean.empty() ? nullptr : c.mean.data();
    o->mean_dim = (int)c.mean.size();
    o->stats_var = c.var.empty() ? nullptr : c.var.data();
    o->var_dim = (int)c.var.size();
    o->count = c.count;
    o->epsilon = c.eps;
    o->target_rms = c.rms;
    o->num_filters_in = c.nfi;
    o->num_filters_out = c.nfo;
    o->height_in = c.hin;
    o->height_out = c.hout;
    o->num_heads = c.heads;
    o->key_dim = c.kdim;
    o->value_dim = c.vdim;
    o->key_scale = c.kscale;
    o->learning_rate = c.lr;
    o->max_change = c.maxc;
    o->l2_regularize = c.l2;
    return 0;
}

}  // extern "C"

// ====================================================================== loading
namespace {

struct Param {
    int rows, cols;
    long long off;
};

struct Loader {
    KfNet *net;
    const KfNnet3Model *m;
    int mode;
    std::map<std::string, Param> params;
    std::vector<float> flat;
    struct Bn {
        std::string layer;
        int which;
        std::vector<float> mean, var, gamma, beta;
        float eps;
    };
    std::vector<Bn> bns;
    struct Idct {
        std::string layer;
        std::vector<float> m;
        int d;
    };
    std::vector<Idct> idcts;
    std::vector<std::pair<std::string, float>> kscales;
    KfLoadStats st{0, 0, 0};

    const Comp *need(const std::string &n) {
        const Comp *c = m->get(n);
        if (!c) set_err("%s not found", n.c_str());
        return c;
    }
    // replaceMatrix / transposeF32 into the flat parameter `pname` ([in x out])
    bool matrix(const std::string &pname, const Comp &c, const char *what) {
        auto it = params.find(pname);
        if (it == params.end()) {
            set_err("%s: no parameter %s", what, pname.c_str());
            return false;
        }
        const Param &p = it->second;
        if (c.linear.empty()) return true;  // replaceMatrix: empty data is a no-op
        if ((long long)c.linear.size() != (long long)c.rows * c.cols) {
            set_err("%s: data %zu != %dx%d", what, c.linear.size(), c.rows, c.cols);
            return false;
        }
        if (c.cols != p.rows || c.rows != p.cols) {
            set_err("%s: Kaldi matrix %dx%d does not match the layer's %dx%d (out x in)", what, c.rows, c.cols,
                    p.cols, p.rows);
            return false;
        }
        for (int r = 0; r < c.rows; ++r)
            for (int k = 0; k < c.cols; ++k) flat[p.off + (long long)k * c.rows + r] = c.linear[(size_t)r * c.cols + k];
        st.params += (long long)c.rows * c.cols;
        return true;
    }
    // replaceVector; an empty bias is zeroed in KF_LOAD_NEW (gpu.ZeroTensor), kept otherwise
    bool vector(const std::string &pname, const std::vector<float> &v, const char *what) {
        auto it = params.find(pname);
        if (it == params.end()) {
            set_err("%s: no parameter %s", what, pname.c_str());
            return false;
        }
        const Param &p = it->second;
        const long long n = (long long)p.rows * p.cols;
        if (v.empty()) {
            if (mode == KF_LOAD_NEW)
                for (long long i = 0; i < n; ++i) flat[p.off + i] = 0.f;
            return true;
        }
        if ((long long)v.size() != n) {
            set_err("%s: bias of %zu values, the layer has %lld", what, v.size(), n);
            return false;
        }
        for (long long i = 0; i < n; ++i) flat[p.off + i] = v[i];
        st.params += n;
        return true;
    }
    // makeBN / makeBlockBN (KF_LOAD_NEW) or replaceBN (KF_LOAD_REPLACE), dim checked
    bool bn(const std::string &layer, int which, const Comp &c, int dim, bool block, const char *what) {
        const int d = (int)c.mean.size();
        if (d == 0) {
            set_err("%s: empty StatsMean", what);
            return false;
        }
        if (d != dim) {
            set_err("%s: %d statistics, the layer needs %d", what, d, dim);
            return false;
        }
        const float rms = c.rms <= 0 ? 1.0f : c.rms;
        const float eps = c.eps <= 0 ? 0.001f : c.eps;
        Bn b{layer, which, std::vector<float>(d), std::vector<float>(d), std::vector<float>(d),
             std::vector<float>(d), eps};
        for (int i = 0; i < d; ++i) {
            const float mu = c.mean[i];
            float v = i < (int)c.var.size() ? c.var[i] : 0.f;
            if (mode == KF_LOAD_REPLACE) {
                if (v < 0) v = 0;
                const float inv = (float)(1.0 / std::sqrt((double)(v + eps)));
                b.mean[i] = mu;
                b.var[i] = v;
                b.gamma[i] = rms * inv;
                b.beta[i] = -mu * b.gamma[i];
            } else {
                if (block && v < 0) v = 0;  // makeBlockBN clamps, makeBN passes the stats through
                if (!block && (int)c.var.size() != d) {
                    set_err("%s: StatsVar has %zu values, StatsMean %d", what, c.var.size(), d);
                    return false;
                }
                b.mean[i] = mu;
                b.var[i] = v;
                b.gamma[i] = rms;
                b.beta[i] = 0.f;
            }
        }
        if (mode == KF_LOAD_REPLACE) st.params += (long long)d * 4;
        bns.push_back(std::move(b));
        return true;
    }
};

}  // namespace

extern "C" int nnet_load_kaldi(KfNet *net, const KfNnet3Model *m, int mode, KfLoadStats *stats) {
    if (!net || !m || (mode != KF_LOAD_NEW && mode != KF_LOAD_REPLACE)) {
        set_err("nnet_load_kaldi: bad arguments");
        return -1;
    }
    Loader L;
    L.net = net;
    L.m = m;
    L.mode = mode;
    const int np = nnet_num_param_tensors(net);
    for (int i = 0; i < np; ++i) {
        char nm[256];
        int r, c;
        long long off;
        if (nnet_param_info(net, i, nm, sizeof(nm), &r, &c, &off) != 0) {
            set_err("nnet_param_info failed");
            return -1;
        }
        L.params[nm] = Param{r, c, off};
    }
    L.flat.resize((size_t)nnet_num_params(net));
    if (nnet_get_params(net, L.flat.data()) != 0) {
        set_err("nnet_get_params: %s", nnet_last_error() ? nnet_last_error() : "failed");
        return -1;
    }
    auto shape = [&](const std::string &p, int &r, int &c) {
        auto it = L.params.find(p);
        r = it == L.params.end() ? 0 : it->second.rows;
        c = it == L.params.end() ? 0 : it->second.cols;
    };
    const int nl = nnet_num_layers(net);
    for (int li = 0; li < nl; ++li) {
        char nm[256];
        int ty, din, dout;
        if (nnet_layer_info(net, li, nm, sizeof(nm), &ty, &din, &dout) != 0) {
            set_err("nnet_layer_info failed");
            return -1;
        }
        const std::string n = nm;
        bool ok = true;
        switch (ty) {
            case NNET_IDCT: {
                const Comp *c = L.need("idct");
                if (!c) return -1;
                if (c->rows != dout || c->cols != din || (int)c->linear.size() != din * dout) {
                    set_err("idct: matrix %dx%d, the layer needs %dx%d", c->rows, c->cols, dout, din);
                    return -1;
                }
                std::vector<float> t((size_t)din * dout);
                for (int r = 0; r < c->rows; ++r)
                    for (int k = 0; k < c->cols; ++k) t[(size_t)k * c->rows + r] = c->linear[(size_t)r * c->cols + k];
                L.idcts.push_back({n, std::move(t), din});
                L.st.params += (long long)din * dout;
                break;
            }
            case NNET_LINEAR: {
                const Comp *c = L.need(n);
                ok = c && L.matrix(n + ".W", *c, n.c_str());
                break;
            }
            case NNET_BATCHNORM: {
                const Comp *c = L.need(n);
                ok = c && L.bn(n, 0, *c, dout, false, n.c_str());
                break;
            }
            case NNET_CONV_RELU_BN: {
                const Comp *cv = L.need(n + ".conv");
                ok = cv && L.matrix(n + ".W", *cv, (n + ".conv").c_str());
                if (ok && !cv->bias.empty()) ok = L.vector(n + ".Bias", cv->bias, (n + ".conv bias").c_str());
                const Comp *b = ok ? L.need(n + ".batchnorm") : nullptr;
                int r, fo;
                shape(n + ".W", r, fo);
                ok = ok && b && L.bn(n, 0, *b, fo, true, (n + ".batchnorm").c_str());
                break;
            }
            case NNET_TDNNF: {
                const Comp *lin = L.need(n + ".linear");
                ok = lin && L.matrix(n + ".LinearW", *lin, (n + ".linear").c_str());
                const Comp *aff = ok ? L.need(n + ".affine") : nullptr;
                ok = ok && aff && L.matrix(n + ".AffineW", *aff, (n + ".affine").c_str());
                ok = ok && L.vector(n + ".AffineBias", aff->bias, (n + ".affine bias").c_str());
                const Comp *b = ok ? L.need(n + ".batchnorm") : nullptr;
                ok = ok && b && L.bn(n, 0, *b, dout, false, (n + ".batchnorm").c_str());
                break;
            }
            case NNET_PREFINAL: {
                const std::string pre = n.find("xent") != std::string::npos ? "prefinal-xent" : "prefinal-chain";
                int r, big, small;
                shape(n + ".BigW", r, big);
                shape(n + ".SmallW", r, small);
                const Comp *aff = L.need(pre + ".affine");
                ok = aff && L.matrix(n + ".BigW", *aff, (pre + ".affine").c_str());
                ok = ok && L.vector(n + ".BigBias", aff->bias, (pre + ".affine bias").c_str());
                const Comp *lin = ok ? L.need(pre + ".linear") : nullptr;
                ok = ok && lin && L.matrix(n + ".SmallW", *lin, (pre + ".linear").c_str());
                const Comp *b1 = ok ? L.need(pre + ".batchnorm1") : nullptr;
                ok = ok && b1 && L.bn(n, 0, *b1, big, false, (pre + ".batchnorm1").c_str());
                if (ok && mode == KF_LOAD_NEW) {
                    const Comp *b2 = m->get(pre + ".batchnorm2");
                    if (b2) ok = L.bn(n, 1, *b2, small, false, (pre + ".batchnorm2").c_str());
                }
                break;
            }
            case NNET_OUTPUT: {
                const Comp *c = L.need(n + ".affine");
                ok = c && L.matrix(n + ".W", *c, (n + ".affine").c_str());
                ok = ok && L.vector(n + ".Bias", c->bias, (n + ".affine bias").c_str());
                break;
            }
            case NNET_ATTENTION: {
                if (mode == KF_LOAD_REPLACE) {  // LoadWeights: "attention loading not implemented"
                    L.st.layers_skipped++;
                    continue;
                }
                // allocWeightsFromKaldi (:221-275): affine, batchnorm, key scale
                const Comp *aff = L.need(n + ".affine");
                ok = aff && L.matrix(n + ".W", *aff, (n + ".affine").c_str());
                ok = ok && L.vector(n + ".Bias", aff->bias, (n + ".affine bias").c_str());
                const Comp *b = ok ? L.need(n + ".batchnorm") : nullptr;
                ok = ok && b && L.bn(n, 0, *b, dout, false, (n + ".batchnorm").c_str());
                const Comp *at = m->get(n + ".attention");
                if (ok && at && at->kscale > 0) L.kscales.emplace_back(n, at->kscale);
                break;
            }
            default:
                L.st.layers_skipped++;
                continue;
        }
        if (!ok) return -1;
        L.st.layers_loaded++;
    }
    // every check passed: apply
    if (nnet_set_params(net, L.flat.data()) != 0) {
        set_err("nnet_set_params: %s", nnet_last_error() ? nnet_last_error() : "failed");
        return -1;
    }
    for (auto &b : L.bns)
        if (nnet_set_bn(net, b.layer.c_str(), b.which, b.mean.data(), b.var.data(), b.gamma.data(), b.beta.data(),
                        b.eps, 1.0f) != 0) {
            set_err("nnet_set_bn %s: %s", b.layer.c_str(), nnet_last_error() ? nnet_last_error() : "failed");
            return -1;
        }
    for (auto &i : L.idcts)
        if (nnet_set_idct(net, i.layer.c_str(), i.m.data(), i.d, i.d) != 0) {
            set_err("nnet_set_idct: %s", nnet_last_error() ? nnet_last_error() : "failed");
            return -1;
        }
    for (auto &k : L.kscales)
        if (nnet_set_key_scale(net, k.first.c_str(), k.second) != 0) {
            set_err("nnet_set_key_scale: %s", nnet_last_error() ? nnet_last_error() : "failed");
            return -1;
        }
    if (stats) *stats = L.st;
    return 0;
}
