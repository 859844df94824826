// nnet_host.h — internal types of the C++ host layer (restating internal/nnet).
#pragma once
#include <map>
#include <string>
#include <vector>

#include "../../include/bridge.h"
#include "../../include/kf_dp.h"
#include "../../include/kf_nnet.h"
#include "../../include/kf_ops.h"
#include "../../include/ops.h"

namespace kf {

// xconfig.go:18-30 (same order as NNET_* codes)
enum class LayerType {
    Input = 0, IDCT, Linear, Batchnorm, SpecAugment, CombineFeatureMaps, ConvReluBN, TDNNF,
    Attention, Prefinal, Output
};

struct LayerConfig {  // xconfig.go:68-74
    LayerType type = LayerType::Input;
    std::string name;
    std::map<std::string, std::string> params;
    int line = 0;
    std::string get(const std::string &k, const std::string &def) const;
    int get_int(const std::string &k, int def) const;
    double get_float(const std::string &k, double def) const;
    bool get_bool(const std::string &k, bool def) const;
    std::vector<int> get_ints(const std::string &k) const;
};

struct InputRef {  // xconfig.go:279-293
    enum Kind { Simple, Append, Replace, Previous } kind = Previous;
    std::string name;
    std::vector<std::string> names;
};

struct Layer {  // layers.go:12-120 (specs flattened)
    LayerConfig cfg;
    std::string name;
    LayerType type = LayerType::Input;
    int in_dim = 0, out_dim = 0;
    InputRef input;
    std::vector<std::string> input_names;
    // idct / batchnorm
    double cepstral_lifter = 22, target_rms = 1.0;
    // combine-feature-maps
    int height = 0, nf1 = 1, nf2 = 1;
    // conv
    int hin = 0, hout = 0, hsub = 1, fin = 0, fout = 0;
    std::vector<int> time_offsets, height_offsets;
    // tdnnf
    int bottleneck = 0, time_stride = 3;
    double bypass_scale = 0.66;
    // prefinal
    int small_dim = 0, big_dim = 0;
    // output
    bool include_log_softmax = true;
    // attention-relu-batchnorm (layers.go:298-321, AttentionSpec :92-104)
    int num_heads = 1, key_dim = 0, value_dim = 0, num_left = 0, num_right = 0, att_stride = 1;
    double key_scale = 0;  // 0 -> 1/sqrt(key_dim) (weight_loader.go:266-271)
};

bool ParseXConfig(const std::string &text, std::vector<LayerConfig> &out, std::string &err);
InputRef ParseInput(const std::string &spec);
bool ResolveLayers(const std::vector<LayerConfig> &cfgs, std::vector<Layer> &layers,
                   std::string &err);

}  // namespace kf
