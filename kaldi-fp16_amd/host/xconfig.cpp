// xconfig.cpp — Kaldi xconfig parsing and layer resolution, restating the
// reference's internal/nnet/xconfig.go:143-325 and internal/nnet/layers.go:126-374
// in C++ (the reference's host language, Go, is not available in this image).
#include "nnet_host.h"

#include <cstdio>
#include <cstdlib>
#include <sstream>

namespace kf {

static const std::map<std::string, LayerType> kTypeFromString = {
    {"input", LayerType::Input},
    {"idct-layer", LayerType::IDCT},
    {"linear-component", LayerType::Linear},
    {"batchnorm-component", LayerType::Batchnorm},
    {"spec-augment-layer", LayerType::SpecAugment},
    {"combine-feature-maps-layer", LayerType::CombineFeatureMaps},
    {"conv-relu-batchnorm-layer", LayerType::ConvReluBN},
    {"tdnnf-layer", LayerType::TDNNF},
    {"attention-relu-batchnorm-layer", LayerType::Attention},
    {"prefinal-layer", LayerType::Prefinal},
    {"output-layer", LayerType::Output},
};

std::string LayerConfig::get(const std::string &k, const std::string &def) const {
    auto it = params.find(k);
    return it == params.end() ? def : it->second;
}
int LayerConfig::get_int(const std::string &k, int def) const {
    auto it = params.find(k);
    if (it == params.end()) return def;
    char *end = nullptr;
    long v = strtol(it->second.c_str(), &end, 10);
    return (end && *end == 0 && !it->second.empty()) ? (int)v : def;  // strconv.Atoi
}
double LayerConfig::get_float(const std::string &k, double def) const {
    auto it = params.find(k);
    if (it == params.end()) return def;
    char *end = nullptr;
    double v = strtod(it->second.c_str(), &end);
    return (end && *end == 0 && !it->second.empty()) ? v : def;
}
bool LayerConfig::get_bool(const std::string &k, bool def) const {
    auto it = params.find(k);
    if (it == params.end()) return def;
    std::string v;
    for (char c : it->second) v += (char)tolower(c);
    if (v == "true" || v == "1" || v == "yes") return true;
    if (v == "false" || v == "0" || v == "no") return false;
    return def;
}
std::vector<int> LayerConfig::get_ints(const std::string &k) const {
    std::vector<int> r;
    auto it = params.find(k);
    if (it == params.end() || it->second.empty()) return r;
    std::stringstream ss(it->second);
    std::string part;
    while (std::getline(ss, part, ',')) {
        size_t a = part.find_first_not_of(" \t"), b = part.find_last_not_of(" \t");
        if (a == std::string::npos) continue;
        std::string p = part.substr(a, b - a + 1);
        char *end = nullptr;
        long v = strtol(p.c_str(), &end, 10);
        if (end && *end == 0) r.push_back((int)v);
    }
    return r;
}

// xconfig.go:242-271 — split on blanks outside parentheses
static std::vector<std::string> tokenize(const std::string &line) {
    std::vector<std::string> toks;
    std::string cur;
    int depth = 0;
    for (char ch : line) {
        if (ch == '(') {
            depth++;
            cur += ch;
        } else if (ch == ')') {
            depth--;
            cur += ch;
        } else if (ch == ' ' || ch == '\t') {
            if (depth > 0) cur += ch;
            else if (!cur.empty()) {
                toks.push_back(cur);
                cur.clear();
            }
        } else {
            cur += ch;
        }
    }
    if (!cur.empty()) toks.push_back(cur);
    return toks;
}

// xconfig.go:159-236
bool ParseXConfig(const std::string &text, std::vector<LayerConfig> &out, std::string &err) {
    std::stringstream ss(text);
    std::string raw;
    int lineno = 0;
    while (std::getline(ss, raw)) {
        lineno++;
        size_t a = raw.find_first_not_of(" \t\r"), b = raw.find_last_not_of(" \t\r");
        if (a == std::string::npos) continue;
        std::string line = raw.substr(a, b - a + 1);
        if (line[0] == '#') continue;
        auto toks = tokenize(line);
        if (toks.empty()) continue;
        auto it = kTypeFromString.find(toks[0]);
        if (it == kTypeFromString.end()) {
            err = "line " + std::to_string(lineno) + ": unknown layer type: \"" + toks[0] + "\"";
            return false;
        }
        LayerConfig lc;
        lc.type = it->second;
        lc.line = lineno;
        for (size_t i = 1; i < toks.size(); ++i) {
            size_t eq = toks[i].find('=');
            if (eq == std::string::npos) continue;  // unexpanded $vars are skipped
            lc.params[toks[i].substr(0, eq)] = toks[i].substr(eq + 1);
        }
        lc.name = lc.get("name", "");
        if (lc.name.empty() && lc.type != LayerType::Input) {
            err = "line " + std::to_string(lineno) + ": layer missing name";
            return false;
        }
        if (lc.type == LayerType::Input && lc.name.empty())
            lc.name = "input_" + std::to_string(lineno);
        out.push_back(lc);
    }
    return true;
}

// xconfig.go:296-325
InputRef ParseInput(const std::string &spec_in) {
    InputRef r;
    size_t a = spec_in.find_first_not_of(" \t"), b = spec_in.find_last_not_of(" \t");
    std::string spec = a == std::string::npos ? "" : spec_in.substr(a, b - a + 1);
    if (spec.empty()) {
        r.kind = InputRef::Previous;
        return r;
    }
    auto trim = [](std::string s) {
        size_t x = s.find_first_not_of(" \t"), y = s.find_last_not_of(" \t");
        return x == std::string::npos ? std::string() : s.substr(x, y - x + 1);
    };
    if (spec.rfind("Append(", 0) == 0 && spec.back() == ')') {
        std::string inner = spec.substr(7, spec.size() - 8);
        std::stringstream ss(inner);
        std::string part;
        while (std::getline(ss, part, ',')) r.names.push_back(trim(part));
        r.kind = InputRef::Append;
        return r;
    }
    if (spec.rfind("ReplaceIndex(", 0) == 0 && spec.back() == ')') {
        std::string inner = spec.substr(13, spec.size() - 14);
        r.kind = InputRef::Replace;
        r.name = trim(inner.substr(0, inner.find(',')));
        return r;
    }
    r.kind = InputRef::Simple;
    r.name = spec;
    return r;
}

// layers.go:357-374 — exact name, else the latest "name.suffix" layer
static const Layer *resolve_name(const std::string &name, const std::vector<Layer> &layers) {
    const Layer *best = nullptr;
    for (const auto &l : layers) {
        if (l.name == name) return &l;
    }
    for (const auto &l : layers) {
        if (l.name.size() > name.size() && l.name.compare(0, name.size(), name) == 0 &&
            l.name[name.size()] == '.') {
            if (!best || l.cfg.line > best->cfg.line) best = &l;
        }
    }
    return best;
}

// layers.go:126-355
bool ResolveLayers(const std::vector<LayerConfig> &cfgs, std::vector<Layer> &layers,
                   std::string &err) {
    for (size_t idx = 0; idx < cfgs.size(); ++idx) {
        const LayerConfig &cfg = cfgs[idx];
        Layer L;
        L.cfg = cfg;
        L.name = cfg.name;
        L.type = cfg.type;
        L.input = ParseInput(cfg.get("input", ""));
        auto fail = [&](const std::string &m) {
            err = "layer \"" + cfg.name + "\" (line " + std::to_string(cfg.line) + "): " + m;
            return false;
        };
        switch (L.input.kind) {
            case InputRef::Previous:
                if (idx > 0) {
                    L.in_dim = layers[idx - 1].out_dim;
                    L.input_names = {layers[idx - 1].name};
                }
                break;
            case InputRef::Simple:
            case InputRef::Replace: {
                const Layer *src = resolve_name(L.input.name, layers);
                if (!src) return fail("input \"" + L.input.name + "\" not found");
                L.in_dim = src->out_dim;
                L.input_names = {src->name};
                break;
            }
            case InputRef::Append: {
                int tot = 0;
                for (const auto &n : L.input.names) {
                    const Layer *src = resolve_name(n, layers);
                    if (!src) return fail("append input \"" + n + "\" not found");
                    tot += src->out_dim;
                    L.input_names.push_back(src->name);
                }
                L.in_dim = tot;
                break;
            }
        }
        switch (cfg.type) {
            case LayerType::Input: {
                int dim = cfg.get_int("dim", 0);
                if (dim <= 0) return fail("input layer missing dim");
                L.in_dim = L.out_dim = dim;
                break;
            }
            case LayerType::IDCT:
                L.out_dim = cfg.get_int("dim", L.in_dim);
                L.cepstral_lifter = cfg.get_float("cepstral-lifter", 22);
                break;
            case LayerType::Linear: {
                int dim = cfg.get_int("dim", 0);
                if (dim <= 0) return fail("linear-component missing dim");
                L.out_dim = dim;
                break;
            }
            case LayerType::Batchnorm:
                L.out_dim = L.in_dim;
                L.target_rms = cfg.get_float("target-rms", 1.0);
                break;
            case LayerType::SpecAugment:
                L.out_dim = L.in_dim;
                break;
            case LayerType::CombineFeatureMaps:
                L.height = cfg.get_int("height", 0);
                L.nf1 = cfg.get_int("num-filters1", 1);
                L.nf2 = cfg.get_int("num-filters2", 1);
                L.out_dim = L.in_dim;
                break;
            case LayerType::ConvReluBN: {
                L.hin = cfg.get_int("height-in", 0);
                L.hout = cfg.get_int("height-out", L.hin);
                L.hsub = cfg.get_int("height-subsample-out", 1);
                L.fout = cfg.get_int("num-filters-out", 0);
                L.time_offsets = cfg.get_ints("time-offsets");
                L.height_offsets = cfg.get_ints("height-offsets");
                L.fin = L.hin > 0 ? L.in_dim / L.hin : 0;
                L.out_dim = L.hout * L.fout;
                break;
            }
            case LayerType::TDNNF: {
                int dim = cfg.get_int("dim", 0), bn = cfg.get_int("bottleneck-dim", 0);
                if (dim <= 0 || bn <= 0) return fail("tdnnf-layer missing dim or bottleneck-dim");
                L.out_dim = dim;
                L.bottleneck = bn;
                L.time_stride = cfg.get_int("time-stride", 3);
                L.bypass_scale = cfg.get_float("bypass-scale", 0.66);
                break;
            }
            case LayerType::Attention: {
                int nh = cfg.get_int("num-heads", 1), vd = cfg.get_int("value-dim", 0);
                int ctx = 1 + cfg.get_int("num-left-inputs", 0) + cfg.get_int("num-right-inputs", 0);
                L.out_dim = nh * (vd + ctx);
                L.num_heads = nh;
                L.value_dim = vd;
                L.key_dim = cfg.get_int("key-dim", 0);
                L.num_left = cfg.get_int("num-left-inputs", 0);
                L.num_right = cfg.get_int("num-right-inputs", 0);
                L.att_stride = cfg.get_int("time-stride", 1);
                L.key_scale = cfg.get_float("key-scale", 0.0);
                break;
            }
            case LayerType::Prefinal: {
                int sm = cfg.get_int("small-dim", 0), bg = cfg.get_int("big-dim", 0);
                if (sm <= 0 || bg <= 0) return fail("prefinal-layer missing small-dim or big-dim");
                L.small_dim = sm;
                L.big_dim = bg;
                L.out_dim = sm;
                break;
            }
            case LayerType::Output: {
                int dim = cfg.get_int("dim", 0);
                if (dim <= 0) return fail("output-layer missing dim");
                L.out_dim = dim;
                L.include_log_softmax = cfg.get_bool("include-log-softmax", true);
                break;
            }
        }
        layers.push_back(L);
    }
    return true;
}

}  // namespace kf
