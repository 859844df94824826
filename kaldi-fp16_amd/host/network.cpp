// network.cpp — Network / backward / SGD of the C++ host layer.
//
// Restates internal/nnet/forward.go (Network.Forward and the per-layer
// forward functions), internal/nnet/network_backward.go (Network.Backward) and
// internal/gpu/optimize.go (SGDOptimizer) on top of the MI355X C-ABI:
//   * every dense product is one kf_gemm_fused / kf_gemm_wgrad launch whose
//     operand addressing does the TDNN splice (forward.go:699-790) and the conv
//     im2col (forward.go:435-456) implicitly, with bias / ReLU / BatchNorm /
//     bypass fused into the epilogue;
//   * backward is the exact gradient of that forward (the reference's
//     backwardTDNNF / backwardPrefinal are not);
//   * all trainable parameters live in one flat fp32 master / fp16 working /
//     fp32 gradient / fp32 velocity allocation, so the optimiser is one launch
//     and the data-parallel gradient exchange is one contiguous buffer.
// Memory comes from the bridge_* ABI, as the Go layer does (internal/gpu/tensor.go).
#include <algorithm>
#include <climits>
#include <cstdlib>
#include <cmath>
#include <functional>
#include <cstdio>
#include <cstring>
#include <memory>

#include "nnet_host.h"

using kf::Layer;
using kf::LayerType;

static __thread char g_nnet_err[1024];
static void set_err(const std::string &s) { snprintf(g_nnet_err, sizeof g_nnet_err, "%s", s.c_str()); }
extern "C" const char *nnet_last_error(void) { return g_nnet_err[0] ? g_nnet_err : nullptr; }

namespace {

struct ParamRef {
    std::string name;
    int rows, cols;
    long long off;
};

// an MXFP8 tensor: e4m3 [rows x ld] + E8M0 scales [rows x ld/32] (kf_ops.h)
struct Mx {
    uint8_t *q = nullptr, *s = nullptr;
    int ld = 0;
};

struct NetLayer {
    Layer L;
    int input = -1;  // index into layers, -1 = network input (features)
    int pW = -1, pb = -1, pW2 = -1, pb2 = -1;
    std::vector<int> dt, dh;  // conv: cross product of offsets (Kaldi)
    float *bn_scale = nullptr, *bn_shift = nullptr;    // device, expanded to out width
    float *bn2_scale = nullptr, *bn2_shift = nullptr;  // prefinal small BN
    std::vector<float> hbn[4], hbn2[4];                // host mean,var,gamma,beta
    float bn_eps = 1e-3f, bn_rms = 1.f, bn2_eps = 1e-3f, bn2_rms = 1.f;
    bool has_bn2 = false;
    void *act = nullptr;      // fp16 [maxT x out_dim] (or alias of the input for spec-augment)
    bool act_alias = false;
    uint8_t *mask = nullptr;  // relu bits
    void *aux = nullptr;      // tdnnf bottleneck / prefinal big
    void *idct = nullptr;     // fp16 [D x D]
    void *dproj = nullptr;    // attention: fp16 [maxT x affine] gradient of aux (the affine output)
    float *att_scratch = nullptr;  // attention: fp32 [2 x maxT x heads x context]
    float key_scale = 0.f;
    bool per_seq = false;     // runs on the B per-sequence rows (ReplaceIndex(ivector, t, 0) branch)
    int input2 = -100;        // combine-feature-maps: second Append input (-2 = ivector input)
    // small num-filters-in conv (fin not 1 and not a multiple of 32): im2col + GEMM
    int kp = 0;               // padded K (multiple of 64)
    void *im2col = nullptr;   // fp16 [maxT*hout x kp], also reused for dP in backward
    void *wpad = nullptr;     // fp16 [kp x fout], rows >= ntaps*fin zero
    float *gwpad = nullptr;   // fp32 [kp x fout] weight gradient over the padded K
    void *gdb = nullptr;      // fp16 per-sequence gradient [maxT x dim] (combine backward)
    bool bypass = false;
    bool needs_dx = false;
    bool compact = false;     // computed on the supervised row set (nnet_set_row_subsampling)
    // MXFP8 forward (nnet_set_fp8): output / aux copies written by the producing
    // GEMM epilogue, and the weights quantised [N][K] with each splice part padded
    Mx a8, x8, w8, w8b;
    // MXFP8 train step, TDNN-F with a time stride: the affine weight rows for the input
    // gradient, [bottleneck x 2 * pad128(out_dim)] (part p = rows p*bn .. of W2, blocks of 32
    // along out_dim), quantised with the forward copies
    Mx w8d;
    // k-contiguous (transposed) fp16 copy of a short-K forward weight, [N x K], for the
    // fused GEMM's k-contiguous B; refreshed from w16 before a forward after any change
    void *wt = nullptr;
    int wt_pi = -1, wt_K = 0, wt_N = 0;
    // strided conv (height-subsample-out > 1), input gradient as one GEMM over every residue:
    // the merged weight rows [np * hsub * fin x fout] (block (p, pi) = tap wm_map[p*hsub+pi]'s
    // fin rows of W, or zeros), the parts' (dt, dh') in wm_dt / wm_dh
    void *wm = nullptr;
    int wm_np = -1;
    // conv input gradient, per-tap transposed weight blocks [fout x fin] (dgrad_wt)
    void *wtd = nullptr;
    std::vector<int> wm_map, wm_dt, wm_dh;
};

inline size_t align_up(size_t v, size_t a) { return (v + a - 1) / a * a; }

KfAttention att_args(const NetLayer &nl, int T) {
    const Layer &L = nl.L;
    KfAttention a;
    a.proj = nl.aux;
    a.T = T;
    a.num_heads = L.num_heads;
    a.key_dim = L.key_dim;
    a.value_dim = L.value_dim;
    a.context = 1 + L.num_left + L.num_right;
    a.ldp = (long long)L.num_heads * (2 * L.key_dim + L.value_dim + a.context);
    a.num_left = L.num_left;
    a.stride = L.att_stride;
    a.key_scale = nl.key_scale;
    return a;
}

KfOperand op_base(const void *p, long long ld, int rows, int cols, int kcontig) {
    KfOperand d;
    memset(&d, 0, sizeof d);
    d.base = p;
    d.ld = ld;
    d.nrows = rows;
    d.ncols = cols;
    d.kcontig = kcontig;
    d.nparts = 1;
    d.part_width = cols;
    d.T = rows;
    d.hout = 1;
    d.hsrc = 1;
    d.hmul = 0;
    d.hdiv = 1;
    d.tpolicy = KF_ZERO;
    for (int i = 0; i < KF_MAX_PARTS; ++i) d.edge_t[i] = -1;
    return d;
}
// [x(t+dt0) | x(t+dt1)] over T rows of width d (forward.go:699-790)
KfOperand op_splice(const void *p, int T, int d, int dt0, int dt1, int policy, int kcontig) {
    KfOperand o = op_base(p, d, T, 2 * d, kcontig);
    o.nparts = 2;
    o.part_width = d;
    o.dt[0] = dt0;
    o.dt[1] = dt1;
    o.tpolicy = policy;
    return o;
}
// im2col of a conv layer input [T x hin*fin] -> rows (t,h) < T*hout, cols (o,f)
KfOperand op_im2col(const NetLayer &nl, const void *x, int T, int kcontig) {
    const Layer &L = nl.L;
    const int noff = (int)nl.dt.size();
    KfOperand o = op_base(x, (long long)L.hin * L.fin, T * L.hout, noff * L.fin, kcontig);
    o.nparts = noff;
    o.part_width = L.fin;
    o.T = T;
    o.hout = L.hout;
    o.hsrc = L.hin;
    o.hmul = L.hsub;
    o.hdiv = 1;
    o.tpolicy = KF_ZERO;
    for (int i = 0; i < noff; ++i) {
        o.dt[i] = nl.dt[i];
        o.dh[i] = nl.dh[i];
    }
    return o;
}
// transpose-conv gather of dz [(t,h) x fout]: rows (t',h') < T*hin, cols (o,n)
KfOperand op_col2im(const NetLayer &nl, const void *dz, int T) {
    const Layer &L = nl.L;
    const int noff = (int)nl.dt.size();
    KfOperand o = op_base(dz, (long long)L.hout * L.fout, T * L.hin, noff * L.fout, 1);
    o.nparts = noff;
    o.part_width = L.fout;
    o.T = T;
    o.hout = L.hin;
    o.hsrc = L.hout;
    o.hmul = 1;
    o.hdiv = L.hsub;
    o.tpolicy = KF_ZERO;
    for (int i = 0; i < noff; ++i) {
        o.dt[i] = -nl.dt[i];
        o.dh[i] = -nl.dh[i];
    }
    return o;
}
// weights W[nparts*rows x width] read as B'[j][(p, n)] = W[p*rows + j][n]
KfOperand op_wrows(const void *W, int nparts, int rows, int width) {
    KfOperand o = op_base(W, width, rows, nparts * width, 1);
    o.nparts = nparts;
    o.part_width = width;
    o.T = nparts * rows;
    for (int p = 0; p < nparts; ++p) o.dt[p] = p * rows;
    return o;
}
KfEpilogue epi0() {
    KfEpilogue e;
    memset(&e, 0, sizeof e);
    e.alpha = 1.f;
    return e;
}

}  // namespace

struct KfNet {
    std::vector<Layer> all;
    std::vector<NetLayer> layers;
    // Model.ChainOutput (model.go:271-281): the output layer named "output", else the first
    // output layer; backward is seeded there. Trainable layers off its input path (the xent
    // branch) get no gradient (network_backward.go:110-115): their ranges are zeroed.
    int chain_out = -1;
    std::vector<std::pair<long long, long long>> offpath;  // (float offset, count) in grad
    int feat_dim = 0, max_T = 0, T = 0;
    const void *features = nullptr;
    // ivector input: one row per sequence, frames -> sequences by
    // seq_off (device int[B+1]); layers fed from it run on B rows (per_seq)
    int ivec_dim = 0, B = 0;
    const void *ivec = nullptr;
    int *seq_off = nullptr;
    long long nparams = 0;
    std::vector<ParamRef> params;
    float *master = nullptr, *grad = nullptr, *vel = nullptr;
    void *w16 = nullptr;
    // input-gradient ring (three deep: a step's output gradient is not rewritten until the
    // weight gradients of the step after next have read it)
    void *dz[3] = {nullptr, nullptr, nullptr}, *g[3] = {nullptr, nullptr, nullptr};
    void *dbott = nullptr, *edge = nullptr;
    // Weight gradients run on their own stream (nnet_set_wgrad_stream, default on): a layer's
    // dW GEMMs hang off the input-gradient chain (dz -> dbott -> dz below) and overlap it.
    // dbott cycles through three buffers by backward step, so the next layers' affine input
    // gradients never wait for this layer's linear weight gradient.
    void *dbott2 = nullptr, *dbott3 = nullptr;
    void *wg_stream = nullptr, *ev_go = nullptr, *ev_side = nullptr;
    void *ev_step[3] = {nullptr, nullptr, nullptr};  // end of a backward step's side work (ring)
    void *ev_aux = nullptr;  // side-stream launches main joins on the spot (conv tail rows / window)
    void *hp_stream = nullptr;  // high-priority stream for the input-gradient chain
    int wg_side = 1;
    // Implicit dz (nnet_set_implicit_dz, default off, fp16 step): the input-gradient epilogue
    // that produces a TDNN-F layer's g stores no dz = rne(g * bnscale * mask); the layer's
    // affine weight and input gradients read g through the forward's ReLU mask (masked
    // operands, kf_ops.h) with the BN scale folded into W2 (w2s scratch) or the weight
    // gradient's reduction. One full-width fp16 tensor fewer written per TDNN-F layer, but
    // step-neutral on the MI355X (the linear input gradient's saving is spent
    // by the masked affine input gradient on the same chain), so off by default.
    int implicit_dz = 0;
    int main_aff = -1;             // nnet_debug_backward (tests): -1 = KF_BWD_MAIN_AFF / 0
    // Row-subsampled train step (nnet_set_row_subsampling, r6). The chain objective reads the
    // output on rows 0 (mod 3) only, and every layer from first_c up (TDNN-F with time
    // stride 0 / 3, linear, prefinal, output) maps row t from rows t, t +- 3 of the layer
    // below; with the splices' clamp at T - 1 the rows those outputs depend on are the rows
    // 0 (mod 3) plus a tail of rows T-1, T-4, ... as deep as the layers. Those layers run on
    // that compact set: compact row c is source row 3c for c < Tc0, else
    // (T-1) - 3 (Tc-1-c); a splice of +-3 source rows is +-1 compact row. At the boundary
    // (c = Tc0 - 1 whose +3 row is T-1 = compact Tc-1, and tail row Tc0 whose -3 row is not
    // in the set) the tail row Tc0 is a scratch slot: after each linear GEMM it receives a
    // copy of the bottleneck's row Tc - 1, so row Tc0 - 1's +1 neighbour reads row T-1, and
    // its bottleneck gradient is zeroed after the affine input gradient (its true gradient,
    // as every row outside the set, is zero). Its own values and those its wrong neighbour
    // reaches stay more than the tail's depth away from every row with a gradient.
    int rsub = 0;                  // 3: on
    int first_c = -1;              // lowest compact layer (its input: a conv, full rows)
    // the conv below first_c evaluated on the compact rows only (its output frames 3c and the
    // tail; time-strided halo operand, kf_ops.h KfOperand.tmul): its activation and mask are
    // then in compact rows and first_c reads them directly. Its backward stays on full rows
    // (the input gradient scattered back). KF_RSUB_CONV=0 at nnet_set_row_subsampling: off.
    int conv_c = 0;
    int rs_nt = 0;                 // tail rows when (T - 1) % 3 != 0
    int Tc = 0, Tc0 = 0;           // compact rows of the current forward (0: full rows)
    int maxTc = 0;
    void *xc = nullptr;            // first_c's input, gathered to compact rows
    void *dzc = nullptr;           // first_c's input gradient in compact rows
    uint8_t *mc = nullptr;         // the mask of first_c's input, compact rows
    // bottleneck-gradient row mask [maxTc x rm_bn bits]: all ones but the scratch row Tc0
    // (the TDNN-F affine input gradient zeroes that row in its epilogue)
    uint8_t *rowmask = nullptr;
    int rm_bn = 0, rm_tc0 = -1, rm_tc = -1;
    long long stall_side = 0;      // nnet_debug_backward (tests): spin before side work
    bool dz_imp[3] = {false, false, false};  // dz[i] was left implicit by the producing epilogue
    bool dz_edge[3] = {false, false, false}; // row T of dz[i] already holds the strided TDNN-F edge sum
    void *w2s = nullptr;              // [kaff x dout] fp16: W2 with the BN scale folded in
    void *dbott_last = nullptr;  // the dbott buffer of the last TDNN-F / prefinal step (tests)
    void *dz_last = nullptr;     // the input gradient the last backward step handed down (tests)
    size_t edge_half = 0;
    int fp8 = 0;
    int fp8_dgrad = 1;  // nnet_set_fp8(net, 2): MXFP8 forward, fp16 affine input gradients (tests)
    // MXFP8 copies of dz[0] / dz[1] written by the producing input-gradient epilogue
    // (out8_src = 1) for a TDNN-F layer's affine input gradient, and the layer each holds
    Mx dz8[3];
    int dz8_layer[3] = {-1, -1, -1};
    bool wt_dirty = true;  // the transposed weight copies need a refresh (NetLayer::wt)
    // data parallel (kf_dp.h): gradient buckets exchanged during the backward
    KfDp *dp = nullptr;
    std::vector<int> dp_after;  // bucket j is issued after backward step dp_after[j]
    std::vector<long long> dp_begin, dp_end;
    bool dp_early = false;  // nnet_dp_debug_early: every bucket issued before the backward (tests)
    std::vector<void *> allocs;

    void *dalloc(size_t bytes) {
        void *p = bridge_gpu_malloc(bytes ? bytes : 16);
        if (p) allocs.push_back(p);
        return p;
    }
    ~KfNet() {
        if (wg_stream) bridge_gpu_sync();
        kf_event_free(ev_go);
        kf_event_free(ev_side);
        for (void *e : ev_step) kf_event_free(e);
        kf_event_free(ev_aux);
        kf_stream_free(wg_stream);
        kf_stream_free(hp_stream);
        for (void *p : allocs) bridge_gpu_free(p);
    }
};

namespace {

inline void *wptr(KfNet *net, int pi) {
    return pi < 0 ? nullptr : (char *)net->w16 + net->params[pi].off * 2;
}
inline float *gptr(KfNet *net, int pi) { return pi < 0 ? nullptr : net->grad + net->params[pi].off; }

bool ck(int rc, const char *what) {
    if (rc != 0) {
        const char *e = kf_last_error();
        if (!e) e = kf_layers_last_error();
        if (!e) e = ops_last_error();
        set_err(std::string(what) + ": " + (e ? e : "failed"));
        return false;
    }
    return true;
}

// a network from nnet_create_layout has no device storage
bool on_device(const KfNet *net, const char *what) {
    if (net && net->master) return true;
    set_err(std::string(what) + ": " + (net ? "layout-only network (nnet_create_layout)" : "null network"));
    return false;
}

// makeIDCTMatrix, forward.go:1190-1210
std::vector<float> idct_matrix(int dim, double lifter) {
    std::vector<float> m((size_t)dim * dim);
    for (int i = 0; i < dim; ++i)
        for (int j = 0; j < dim; ++j) {
            double v = cos(M_PI * j * (i + 0.5) / dim);
            v *= j == 0 ? sqrt(1.0 / dim) : sqrt(2.0 / dim);
            if (lifter > 0 && j > 0) v *= 1.0 + (lifter / 2.0) * sin(M_PI * j / lifter);
            m[(size_t)i * dim + j] = (float)v;
        }
    return m;
}

// truncating fp32 -> fp16, internal/gpu/tensor.go:158-173 (weights enter this way)
uint16_t f32_to_f16_trunc(float f) {
    uint32_t bits;
    memcpy(&bits, &f, 4);
    uint16_t sign = (uint16_t)((bits >> 16) & 0x8000u);
    int exp = (int)((bits >> 23) & 0xFF) - 127;
    uint32_t frac = bits & 0x7FFFFFu;
    if (exp > 15) return sign | 0x7C00u;
    if (exp < -14) return sign;
    return (uint16_t)(sign | (uint16_t)((exp + 15) << 10) | (uint16_t)(frac >> 13));
}
float f16_to_f32(uint16_t h) {
    uint32_t sign = (uint32_t)(h & 0x8000u) << 16, exp = (h >> 10) & 0x1Fu, frac = h & 0x3FFu;
    uint32_t bits;
    if (exp == 0) {
        if (frac == 0) bits = sign;
        else {
            exp = 1;
            while (!(frac & 0x400u)) {
                frac <<= 1;
                exp--;
            }
            frac &= 0x3FFu;
            bits = sign | ((uint32_t)(127 - 15 + (int)exp) << 23) | (frac << 13);
        }
    } else if (exp == 31) {
        bits = sign | 0x7F800000u | (frac << 13);
    } else {
        bits = sign | ((exp - 15 + 127) << 23) | (frac << 13);
    }
    float f;
    memcpy(&f, &bits, 4);
    return f;
}

int add_param(KfNet *net, const std::string &name, int rows, int cols) {
    ParamRef p{name, rows, cols, net->nparams};
    net->params.push_back(p);
    net->nparams += (long long)align_up((size_t)rows * cols, 64);
    return (int)net->params.size() - 1;
}

// fold frozen BN into per-column scale/shift, expanded to `width` columns by
// repeating the `dim` pattern (conv layers: width = hout*fout, dim = fout)
bool upload_bn(KfNet *net, const std::vector<float> *h, float eps, float rms, int dim, int width,
               float *&dscale, float *&dshift) {
    std::vector<float> sc(width), sh(width);
    for (int c = 0; c < width; ++c) {
        int d = c % dim;
        float inv = 1.0f / sqrtf(h[1][d] + eps);
        float s = rms != 1.0f ? rms * inv : h[2][d] * inv;
        sc[c] = s;
        sh[c] = (rms != 1.0f ? 0.f : h[3][d]) - h[0][d] * s;
    }
    if (!dscale) {
        dscale = (float *)net->dalloc(width * 4);
        dshift = (float *)net->dalloc(width * 4);
        if (!dscale || !dshift) return false;
    }
    return bridge_transfer_float32(dscale, sc.data(), width) == 0 &&
           bridge_transfer_float32(dshift, sh.data(), width) == 0;
}

void identity_bn(std::vector<float> *h, int dim) {  // identityBN, forward.go:1172-1187
    h[0].assign(dim, 0.f);
    h[1].assign(dim, 1.f);
    h[2].assign(dim, 1.f);
    h[3].assign(dim, 0.f);
}

bool is_trainable(LayerType t) {
    return t == LayerType::ConvReluBN || t == LayerType::TDNNF || t == LayerType::Linear ||
           t == LayerType::Prefinal || t == LayerType::Output || t == LayerType::Attention;
}

// affine width of an attention layer: heads x (key + value + query key + query context)
int att_affine(const Layer &L) {
    const int ctx = 1 + L.num_left + L.num_right;
    return L.num_heads * (2 * L.key_dim + L.value_dim + ctx);
}


}  // namespace

// Parse, resolve and lay out the network on the host: layers, inputs, the flat
// parameter layout, the backward path. No device work (nnet_create_layout).
// device = false (nnet_create_layout): the MI355X kernels' shape constraints (dims that
// are multiples of 8 / 32, IDCT <= 64) are not enforced; the layout does not depend on them.
static bool build_topology(KfNet *net, const char *xconfig_text, int max_frames, bool device) {
    std::vector<kf::LayerConfig> cfgs;
    std::string err;
    if (!kf::ParseXConfig(xconfig_text ? xconfig_text : "", cfgs, err) ||
        !kf::ResolveLayers(cfgs, net->all, err)) {
        set_err("parse xconfig: " + err);
        return false;
    }
    if (max_frames <= 0) {
        set_err("max_frames must be positive");
        return false;
    }
    net->max_T = max_frames;
    std::map<std::string, int> index;  // layer name -> index in net->layers (-1 = input)
    for (const Layer &L : net->all) {
        if (L.type == LayerType::Input) {
            if (L.name == "ivector") {  // per-sequence input (Kaldi's ivector-dim input)
                if (net->ivec_dim) {
                    set_err("more than one ivector input");
                    return false;
                }
                net->ivec_dim = L.out_dim;
                index[L.name] = -2;
                continue;
            }
            if (net->feat_dim) {
                set_err("more than one frame-level input layer (only 'input' and 'ivector' are supported)");
                return false;
            }
            net->feat_dim = L.out_dim;
            index[L.name] = -1;
            continue;
        }
        NetLayer nl;
        nl.L = L;
        auto is_seq = [&](int idx) { return idx == -2 || (idx >= 0 && net->layers[idx].per_seq); };
        auto dim_of = [&](int idx) {
            return idx == -2 ? net->ivec_dim : idx >= 0 ? net->layers[idx].L.out_dim : net->feat_dim;
        };
        if (L.input.kind == kf::InputRef::Append && L.type != LayerType::CombineFeatureMaps) {
            // General Append(a, b, ...) (forward.go:264-310: column concat of the inputs, in
            // order; network_backward.go:147-170 splits the gradient back). Each further
            // part is appended by a hidden combine-feature-maps node of height 1, which
            // is exactly a column concat [a | b] with b broadcast to the frames of its
            // sequence when b is per-sequence (an ivector given per frame is B = T
            // sequences of one frame: the reference's [T x dim] ivector Append).
            if (L.input_names.size() < 2) {
                set_err("layer " + L.name + ": Append needs two or more inputs");
                return false;
            }
            std::vector<int> parts;
            for (const auto &nm : L.input_names) {
                auto it = index.find(nm);
                if (it == index.end()) {
                    set_err("layer " + L.name + ": Append input " + nm + " not found");
                    return false;
                }
                parts.push_back(it->second);
            }
            if (is_seq(parts[0])) {
                set_err("layer " + L.name + ": the first Append input must be frame-level");
                return false;
            }
            int cur = parts[0];
            for (size_t k = 1; k < parts.size(); ++k) {
                NetLayer hc;
                hc.L.type = LayerType::CombineFeatureMaps;
                hc.L.name = L.name + ".append" + (parts.size() > 2 ? std::to_string(k) : std::string());
                hc.L.height = 1;
                hc.L.nf1 = dim_of(cur);
                hc.L.nf2 = dim_of(parts[k]);
                hc.L.in_dim = hc.L.out_dim = hc.L.nf1 + hc.L.nf2;
                hc.L.input.kind = kf::InputRef::Append;
                hc.input = cur;
                hc.input2 = parts[k];
                net->layers.push_back(hc);
                index[hc.L.name] = cur = (int)net->layers.size() - 1;
            }
            nl.L.input.kind = kf::InputRef::Simple;
            nl.L.input_names = {net->layers[cur].L.name};
        }
        if (nl.L.input.kind == kf::InputRef::Append) {
            // only combine-feature-maps takes an Append, of a frame-level and a per-sequence
            // (or frame-level) input (Kaldi's Append(idct-batchnorm, ivector-batchnorm))
            if (L.type != LayerType::CombineFeatureMaps || L.input_names.size() != 2) {
                set_err("layer " + L.name + ": Append is supported as the input of combine-feature-maps, of two layers");
                return false;
            }
            auto a = index.find(L.input_names[0]), b = index.find(L.input_names[1]);
            if (a == index.end() || b == index.end() || is_seq(a->second)) {
                set_err("layer " + L.name + ": Append inputs not found, or the first one is per-sequence");
                return false;
            }
            nl.input = a->second;
            nl.input2 = b->second;
        } else {
            if (nl.L.input_names.size() != 1) {
                set_err("layer " + L.name + ": one input expected");
                return false;
            }
            auto it = index.find(nl.L.input_names[0]);
            if (it == index.end()) {
                set_err("layer " + L.name + ": input not found");
                return false;
            }
            nl.input = it->second;
            // ReplaceIndex(x, t, 0) of a per-sequence source, or anything fed by one
            nl.per_seq = is_seq(nl.input);
            if (nl.per_seq && L.type != LayerType::Linear && L.type != LayerType::Batchnorm) {
                set_err("layer " + L.name + ": only linear-component and batchnorm-component run on the "
                        "per-sequence (ivector) branch");
                return false;
            }
        }
        if (L.type == LayerType::CombineFeatureMaps) {
            const int da = nl.input < 0 ? net->feat_dim : net->layers[nl.input].L.out_dim;
            const int db = nl.input2 == -2 ? net->ivec_dim
                           : nl.input2 >= 0 ? net->layers[nl.input2].L.out_dim : net->feat_dim;
            if (nl.input2 == -100 || L.height <= 0 || da != L.height * L.nf1 || db != L.height * L.nf2) {
                set_err("combine-feature-maps " + L.name + ": needs Append(a, b) with dims height*num-filters1 "
                        "and height*num-filters2");
                return false;
            }
        }
        const int din = L.in_dim, dout = L.out_dim;
        const std::string &n = L.name;
        switch (L.type) {
            case LayerType::IDCT:
                if (din != dout || (device && (din > 64 || din % 8))) {
                    set_err("idct-layer " + n + ": dim must equal input dim, <= 64, multiple of 8");
                    return false;
                }
                break;
            case LayerType::Batchnorm:
                identity_bn(nl.hbn, dout);
                nl.bn_rms = (float)L.target_rms;
                break;
            case LayerType::ConvReluBN: {
                if (L.hin <= 0 || L.fin <= 0 || L.fin * L.hin != din || (device && L.fout % 8)) {
                    set_err("conv layer " + n + ": inconsistent height-in / filters");
                    return false;
                }
                for (int a : L.time_offsets)
                    for (int b : L.height_offsets) {
                        nl.dt.push_back(a);
                        nl.dh.push_back(b);
                    }
                if (nl.dt.empty() || nl.dt.size() > KF_MAX_PARTS) {
                    set_err("conv layer " + n + ": need 1..9 (time x height) offsets");
                    return false;
                }
                if (L.fin != 1 && L.fin % 32) {  // small fin: im2col + GEMM (csrc/ivector.hip)
                    nl.kp = (int)((nl.dt.size() * L.fin + 63) / 64 * 64);
                }
                const int K = (int)nl.dt.size() * L.fin;
                nl.pW = add_param(net, n + ".W", K, L.fout);
                nl.pb = add_param(net, n + ".Bias", 1, L.fout);
                identity_bn(nl.hbn, L.fout);
                break;
            }
            case LayerType::TDNNF: {
                const int s = L.time_stride, bn = L.bottleneck;
                if (device && (bn % 32 || din % 32 || dout % 8)) {
                    set_err("tdnnf layer " + n + ": dims must be multiples of 32");
                    return false;
                }
                nl.pW = add_param(net, n + ".LinearW", s > 0 ? 2 * din : din, bn);
                nl.pW2 = add_param(net, n + ".AffineW", s > 0 ? 2 * bn : bn, dout);
                nl.pb2 = add_param(net, n + ".AffineBias", 1, dout);
                nl.bypass = L.bypass_scale > 0 && din == dout;
                identity_bn(nl.hbn, dout);
                break;
            }
            case LayerType::Linear:
                nl.pW = add_param(net, n + ".W", din, dout);
                break;
            case LayerType::Prefinal:
                nl.pW = add_param(net, n + ".BigW", din, L.big_dim);
                nl.pb = add_param(net, n + ".BigBias", 1, L.big_dim);
                nl.pW2 = add_param(net, n + ".SmallW", L.big_dim, L.small_dim);
                identity_bn(nl.hbn, L.big_dim);
                identity_bn(nl.hbn2, L.small_dim);
                nl.has_bn2 = true;
                break;
            case LayerType::Output:
                if (L.include_log_softmax) {
                    // the xent branch (log-softmax output) is a "next" row
                }
                nl.pW = add_param(net, n + ".W", din, dout);
                nl.pb = add_param(net, n + ".Bias", 1, dout);
                break;
            case LayerType::Attention: {
                const int ctx = 1 + L.num_left + L.num_right, A = att_affine(L);
                if (L.num_heads <= 0 || L.key_dim <= 0 || L.value_dim < 0 || L.att_stride <= 0 ||
                    (device && (ctx > 64 || L.num_heads * ctx > 1024 || A % 8 || dout % 8 || din % 8))) {
                    set_err("attention layer " + n + ": needs heads > 0, key-dim > 0, context <= 64, "
                            "heads*context <= 1024 and affine / output / input dims multiples of 8");
                    return false;
                }
                nl.pW = add_param(net, n + ".W", din, A);
                nl.pb = add_param(net, n + ".Bias", 1, A);
                nl.key_scale = L.key_scale > 0 ? (float)L.key_scale : (float)(1.0 / sqrt((double)L.key_dim));
                identity_bn(nl.hbn, dout);
                break;
            }
            case LayerType::SpecAugment:
            case LayerType::CombineFeatureMaps:
                break;
            default:
                set_err("layer " + n + ": type not supported on the MI355X path");
                return false;
        }
        index[L.name] = (int)net->layers.size();
        net->layers.push_back(nl);
    }
    if (net->layers.empty()) {
        set_err("no layers");
        return false;
    }
    for (size_t i = 0; i < net->layers.size() && net->chain_out < 0; ++i)
        if (net->layers[i].L.type == LayerType::Output && net->layers[i].L.name == "output") net->chain_out = (int)i;
    for (size_t i = 0; i < net->layers.size() && net->chain_out < 0; ++i)
        if (net->layers[i].L.type == LayerType::Output) net->chain_out = (int)i;
    if (net->chain_out < 0) net->chain_out = (int)net->layers.size() - 1;
    {
        std::vector<char> on(net->layers.size(), 0);
        for (int cur = net->chain_out; cur >= 0; cur = net->layers[cur].input) on[cur] = 1;
        for (size_t i = 0; i < net->layers.size(); ++i) {
            if (on[i]) continue;
            const NetLayer &nl = net->layers[i];
            for (int pi : {nl.pW, nl.pb, nl.pW2, nl.pb2})
                if (pi >= 0) net->offpath.emplace_back(net->params[pi].off, (long long)net->params[pi].rows * net->params[pi].cols);
        }
    }
    // which layers need an input gradient (a trainable layer lies below them)
    {
        // a trainable layer lies below idx, along inputs and combine-feature-maps' second input
        std::function<bool(int)> below = [&](int idx) -> bool {
            if (idx < 0) return false;
            const NetLayer &q = net->layers[idx];
            return is_trainable(q.L.type) || below(q.input) || (q.input2 >= 0 && below(q.input2));
        };
        for (size_t i = 0; i < net->layers.size(); ++i) net->layers[i].needs_dx = below(net->layers[i].input);
    }
    return true;
}

// Device storage of a laid-out network: parameters, activations, masks, BN, scratch.
static bool alloc_device(KfNet *net, int max_frames) {
    // flat parameter storage
    const long long P = net->nparams > 0 ? net->nparams : 64;
    net->master = (float *)net->dalloc(P * 4);
    net->grad = (float *)net->dalloc(P * 4);
    net->vel = (float *)net->dalloc(P * 4);
    net->w16 = net->dalloc(P * 2);
    if (!net->master || !net->grad || !net->vel || !net->w16) {
        set_err("alloc params: " + std::string(bridge_last_error() ? bridge_last_error() : ""));
        return false;
    }
    bridge_gpu_memset(net->master, 0, P * 4);
    bridge_gpu_memset(net->grad, 0, P * 4);
    bridge_gpu_memset(net->vel, 0, P * 4);
    bridge_gpu_memset(net->w16, 0, P * 2);
    // activations, masks, BN params
    const size_t T = (size_t)max_frames;
    size_t maxw = 16;
    for (auto &nl : net->layers) {
        const Layer &L = nl.L;
        const int dout = L.out_dim;
        maxw = std::max(maxw, (size_t)std::max(L.in_dim, dout));
        if (L.type == LayerType::SpecAugment) {
            nl.act_alias = true;
        } else {
            nl.act = net->dalloc(T * dout * 2);
            if (!nl.act) {
                set_err("alloc activation " + L.name);
                return false;
            }
        }
        int mwidth = 0;
        if (L.type == LayerType::ConvReluBN || L.type == LayerType::TDNNF || L.type == LayerType::Attention)
            mwidth = dout;
        if (L.type == LayerType::Attention) {
            const int A = att_affine(L), ctx = 1 + L.num_left + L.num_right;
            nl.aux = net->dalloc((size_t)T * A * 2);
            nl.dproj = net->dalloc((size_t)T * A * 2);
            nl.att_scratch = (float *)net->dalloc((size_t)2 * T * L.num_heads * ctx * 4);
            if (!nl.aux || !nl.dproj || !nl.att_scratch) {
                set_err("alloc attention buffers");
                return false;
            }
        }
        if (L.type == LayerType::ConvReluBN && nl.kp) {
            nl.im2col = net->dalloc((size_t)T * L.hout * nl.kp * 2);
            nl.wpad = net->dalloc((size_t)nl.kp * L.fout * 2);
            nl.gwpad = (float *)net->dalloc((size_t)nl.kp * L.fout * 4);
            if (!nl.im2col || !nl.wpad || !nl.gwpad) {
                set_err("alloc small-fin conv buffers");
                return false;
            }
            bridge_gpu_memset(nl.wpad, 0, (size_t)nl.kp * L.fout * 2);
        }
        if (L.type == LayerType::CombineFeatureMaps && nl.input2 != -100) {
            nl.gdb = net->dalloc((size_t)T * L.height * L.nf2 * 2);
            if (!nl.gdb) {
                set_err("alloc combine gradient");
                return false;
            }
        }
        if (L.type == LayerType::Prefinal) mwidth = L.big_dim;
        if (mwidth) nl.mask = (uint8_t *)net->dalloc(align_up(T * mwidth / 8 + 16, 256));
        if (L.type == LayerType::TDNNF) nl.aux = net->dalloc(T * L.bottleneck * 2);
        if (L.type == LayerType::Prefinal) {
            nl.aux = net->dalloc(T * L.big_dim * 2);
            maxw = std::max(maxw, (size_t)L.big_dim);
        }
        if (L.type == LayerType::IDCT) {
            auto m = idct_matrix(dout, L.cepstral_lifter);
            std::vector<uint16_t> h(m.size());
            for (size_t i = 0; i < m.size(); ++i) h[i] = f32_to_f16_trunc(m[i]);
            nl.idct = net->dalloc(h.size() * 2);
            if (bridge_transfer_fp16(nl.idct, h.data(), h.size())) {
                set_err("upload idct");
                return false;
            }
        }
        if (L.type == LayerType::Batchnorm &&
            !upload_bn(net, nl.hbn, nl.bn_eps, nl.bn_rms, dout, dout, nl.bn_scale, nl.bn_shift))
            return false;
        if (L.type == LayerType::ConvReluBN &&
            !upload_bn(net, nl.hbn, nl.bn_eps, 1.f, L.fout, dout, nl.bn_scale, nl.bn_shift))
            return false;
        if ((L.type == LayerType::TDNNF || L.type == LayerType::Attention) &&
            !upload_bn(net, nl.hbn, nl.bn_eps, 1.f, dout, dout, nl.bn_scale, nl.bn_shift))
            return false;
        if (L.type == LayerType::Prefinal &&
            (!upload_bn(net, nl.hbn, nl.bn_eps, 1.f, L.big_dim, L.big_dim, nl.bn_scale,
                        nl.bn_shift) ||
             !upload_bn(net, nl.hbn2, nl.bn2_eps, 1.f, L.small_dim, L.small_dim,
                        nl.bn2_scale, nl.bn2_shift)))
            return false;
    }
    // transposed copies of the short-K forward weights (TDNN-F affine, prefinal big)
    for (auto &nl : net->layers) {
        const Layer &L = nl.L;
        int pi = -1, K = 0, N = 0;
        if (L.type == LayerType::TDNNF) {
            pi = nl.pW2;
            K = L.time_stride > 0 ? 2 * L.bottleneck : L.bottleneck;
            N = L.out_dim;
        } else if (L.type == LayerType::Prefinal) {
            pi = nl.pW;
            K = L.in_dim;
            N = L.big_dim;
        }
        if (pi < 0 || K > 512 || K % 32 || N % 32) continue;
        nl.wt = net->dalloc((size_t)K * N * 2);
        if (!nl.wt) {
            set_err("alloc transposed weights " + L.name);
            return false;
        }
        nl.wt_pi = pi;
        nl.wt_K = K;
        nl.wt_N = N;
    }
    // gradient buffers carry two spare rows for the splice-transpose edge sums
    for (int i = 0; i < 3; ++i) {
        net->dz[i] = net->dalloc((T + 2) * maxw * 2);
        net->g[i] = net->dalloc((T + 2) * maxw * 2);
    }
    net->dbott = net->dalloc((T + 2) * maxw * 2);
    net->dbott2 = net->dalloc((T + 2) * maxw * 2);
    net->dbott3 = net->dalloc((T + 2) * maxw * 2);
    {
        size_t w2 = 0;
        for (auto &nl : net->layers)
            if (nl.L.type == LayerType::TDNNF)
                w2 = std::max(w2, (size_t)(nl.L.time_stride > 0 ? 2 : 1) * nl.L.bottleneck * nl.L.out_dim * 2);
        net->w2s = w2 ? net->dalloc(w2) : nullptr;
        if (w2 && !net->w2s) {
            set_err("alloc backward scratch");
            return false;
        }
    }
    net->edge_half = align_up(maxw * 2, 256);
    net->edge = net->dalloc(net->edge_half * 2);
    if (!net->dz[0] || !net->dz[1] || !net->dz[2] || !net->g[0] || !net->g[1] || !net->g[2] || !net->dbott ||
        !net->dbott2 || !net->dbott3 || !net->edge) {
        set_err("alloc backward scratch");
        return false;
    }
    net->wg_stream = kf_stream_new();
    net->hp_stream = kf_stream_new_high();
    net->ev_go = kf_event_new();
    net->ev_side = kf_event_new();
    for (auto &e : net->ev_step) e = kf_event_new();
    net->ev_aux = kf_event_new();
    if (!net->wg_stream || !net->ev_go || !net->ev_side || !net->ev_step[0] || !net->ev_step[1] || !net->ev_step[2] ||
        !net->ev_aux) {
        set_err("create the weight-gradient stream");
        return false;
    }
    return true;
}

extern "C" KfNet *nnet_create(const char *xconfig_text, int max_frames) {
    g_nnet_err[0] = 0;
    std::unique_ptr<KfNet> net(new KfNet);
    if (!build_topology(net.get(), xconfig_text, max_frames, true) || !alloc_device(net.get(), max_frames))
        return nullptr;
    return net.release();
}

extern "C" KfNet *nnet_create_layout(const char *xconfig_text, int max_frames) {
    g_nnet_err[0] = 0;
    std::unique_ptr<KfNet> net(new KfNet);
    if (!build_topology(net.get(), xconfig_text, max_frames, false)) return nullptr;
    return net.release();
}

extern "C" void nnet_free(KfNet *net) {
    kf_take_pending(__func__);
    delete net;
    kf_take_pending("the return of nnet_free");  // a stream / event / free call that failed
}

extern "C" int nnet_num_layers(const KfNet *net) { return (int)net->layers.size(); }

extern "C" int nnet_layer_info(const KfNet *net, int idx, char *name, int namelen, int *type,
                               int *in_dim, int *out_dim) {
    if (idx < 0 || idx >= (int)net->layers.size()) return -1;
    const Layer &L = net->layers[idx].L;
    if (name && namelen > 0) snprintf(name, namelen, "%s", L.name.c_str());
    if (type) *type = (int)L.type;
    if (in_dim) *in_dim = L.in_dim;
    if (out_dim) *out_dim = L.out_dim;
    return 0;
}

extern "C" long long nnet_num_params(const KfNet *net) { return net->nparams; }
extern "C" int nnet_num_param_tensors(const KfNet *net) { return (int)net->params.size(); }
extern "C" int nnet_param_info(const KfNet *net, int idx, char *name, int namelen, int *rows,
                               int *cols, long long *offset) {
    if (idx < 0 || idx >= (int)net->params.size()) return -1;
    const ParamRef &p = net->params[idx];
    if (name && namelen > 0) snprintf(name, namelen, "%s", p.name.c_str());
    if (rows) *rows = p.rows;
    if (cols) *cols = p.cols;
    if (offset) *offset = p.off;
    return 0;
}

static bool quantise_weights(KfNet *net, bool alloc);
extern "C" int nnet_set_params(KfNet *net, const float *host) {
    if (!on_device(net, "set_params")) return -1;
    const long long P = net->nparams;
    std::vector<uint16_t> h(P, 0);
    std::vector<float> m(P, 0.f);
    for (const ParamRef &p : net->params)
        for (long long i = 0; i < (long long)p.rows * p.cols; ++i) {
            uint16_t v = f32_to_f16_trunc(host[p.off + i]);
            h[p.off + i] = v;
            m[p.off + i] = f16_to_f32(v);
        }
    if (bridge_transfer_fp16(net->w16, h.data(), P) || bridge_transfer_float32(net->master, m.data(), P)) {
        set_err(std::string("set_params: ") + (bridge_last_error() ? bridge_last_error() : ""));
        return -1;
    }
    bridge_gpu_memset(net->vel, 0, P * 4);
    net->wt_dirty = true;
    return net->fp8 && !quantise_weights(net, false) ? -1 : 0;
}

extern "C" int nnet_get_params(const KfNet *net, float *host) {
    if (!on_device(net, "get_params")) return -1;
    // D2H through the bridge (fp32 read = 2x fp16 count on a 4-byte aligned buffer)
    std::vector<uint16_t> tmp(net->nparams * 2);
    if (bridge_read_fp16(tmp.data(), net->master, net->nparams * 2)) {
        set_err("get_params");
        return -1;
    }
    memcpy(host, tmp.data(), net->nparams * 4);
    return 0;
}

// Replaces an idct-layer's fixed matrix (LoadWeights / allocWeightsFromKaldi, LayerIDCT:
// weight_loader.go:88-97, :760-770): host fp32 [dim x dim] in the y = x . M orientation,
// stored fp16 by truncation like every weight (tensor.go:158-173).
extern "C" int nnet_set_idct(KfNet *net, const char *layer, const float *m, int rows, int cols) {
    if (!on_device(net, "set_idct")) return -1;
    for (auto &nl : net->layers) {
        if (nl.L.name != layer) continue;
        if (nl.L.type != LayerType::IDCT || !nl.idct) break;
        const int d = nl.L.out_dim;
        if (rows != d || cols != d || !m) {
            set_err("set_idct: " + nl.L.name + " needs a " + std::to_string(d) + "x" + std::to_string(d) +
                    " matrix, got " + std::to_string(rows) + "x" + std::to_string(cols));
            return -1;
        }
        std::vector<uint16_t> h((size_t)d * d);
        for (size_t i = 0; i < h.size(); ++i) h[i] = f32_to_f16_trunc(m[i]);
        if (bridge_transfer_fp16(nl.idct, h.data(), h.size())) {
            set_err("set_idct: upload failed");
            return -1;
        }
        return 0;
    }
    set_err(std::string("set_idct: no idct layer ") + (layer ? layer : "(null)"));
    return -1;
}

// AttentionSpec.KeyScale from a loaded model (weight_loader.go:266-271)
extern "C" int nnet_set_key_scale(KfNet *net, const char *layer, float key_scale) {
    for (auto &nl : net->layers)
        if (nl.L.name == layer && nl.L.type == LayerType::Attention && key_scale > 0) {
            nl.key_scale = key_scale;
            return 0;
        }
    set_err(std::string("set_key_scale: no attention layer ") + (layer ? layer : "(null)"));
    return -1;
}

extern "C" int nnet_set_bn(KfNet *net, const char *layer, int which, const float *mean,
                           const float *var, const float *gamma, const float *beta, float eps,
                           float target_rms) {
    if (!on_device(net, "set_bn")) return -1;
    for (auto &nl : net->layers) {
        if (nl.L.name != layer) continue;
        const Layer &L = nl.L;
        int dim, width;
        std::vector<float> *h;
        // target_rms <= 0: the layer's configured target-rms (batchnorm-component's, else 1)
        if (target_rms <= 0) target_rms = (which != 1 && L.type == LayerType::Batchnorm) ? (float)L.target_rms : 1.0f;
        if (which == 1) {
            if (L.type != LayerType::Prefinal) break;
            dim = width = L.small_dim;
            h = nl.hbn2;
            nl.bn2_eps = eps;
            nl.bn2_rms = target_rms;
        } else {
            if (L.type == LayerType::ConvReluBN) {
                dim = L.fout;
                width = L.out_dim;
            } else if (L.type == LayerType::Prefinal) {
                dim = width = L.big_dim;
            } else if (L.type == LayerType::TDNNF || L.type == LayerType::Batchnorm ||
                       L.type == LayerType::Attention) {
                dim = width = L.out_dim;
            } else {
                break;
            }
            h = nl.hbn;
            nl.bn_eps = eps;
            nl.bn_rms = target_rms;
        }
        h[0].assign(mean, mean + dim);
        h[1].assign(var, var + dim);
        h[2].assign(gamma, gamma + dim);
        h[3].assign(beta, beta + dim);
        if (which == 1) return upload_bn(net, h, eps, target_rms, dim, width, nl.bn2_scale, nl.bn2_shift) ? 0 : -1;
        return upload_bn(net, h, eps, target_rms, dim, width, nl.bn_scale, nl.bn_shift) ? 0 : -1;
    }
    set_err(std::string("set_bn: no BatchNorm '") + std::to_string(which) + "' on layer " + layer);
    return -1;
}

// rows a layer's activations / gradients hold in the current forward
static inline int rows_of(const KfNet *net, int idx) {
    return (idx >= 0 && net->Tc > 0 && net->layers[idx].compact) ? net->Tc : net->T;
}
// the conv below the compact layers, evaluated on the compact rows (KfNet.conv_c)
static inline bool conv_compact(const KfNet *net, int idx) {
    return net->Tc > 0 && net->conv_c && net->first_c >= 0 && idx >= 0 && idx == net->layers[net->first_c].input;
}
// rows a layer's activation holds in the current forward
static inline int act_rows(const KfNet *net, int idx) {
    return conv_compact(net, idx) ? net->Tc : rows_of(net, idx);
}
// strided conv input gradient as one GEMM over every residue (KF_HSUB_MERGE: the largest
// merged width hsub * fin that takes it; default 0 = one GEMM per residue: merged, the zero
// blocks' third more MFMA work cost what the wider tiles gain). The merged
// parts (dt, dh') are ordered by dt, then dh' descending, and taken only when every residue's
// taps then keep their o order. Computed and allocated on first use.
static bool hsub_merge(KfNet *net, NetLayer &nl) {
    const char *e = getenv("KF_HSUB_MERGE");
    const int lim = e ? atoi(e) : 0;
    const Layer &L = nl.L;
    if (L.hsub * L.fin > lim) return false;
    if (nl.wm_np >= 0) return nl.wm_np > 0;
    nl.wm_np = 0;
    const int noff = (int)nl.dt.size(), hs = L.hsub;
    std::vector<std::pair<int, int>> keys;  // (dt, -dh')
    for (int pi = 0; pi < hs; ++pi)
        for (int o = 0; o < noff; ++o) {
            const int r = pi - nl.dh[o];
            if (((r % hs) + hs) % hs) continue;
            keys.push_back({nl.dt[o], -(r / hs)});
        }
    std::sort(keys.begin(), keys.end());
    keys.erase(std::unique(keys.begin(), keys.end()), keys.end());
    const int np = (int)keys.size();
    if (np == 0 || np * hs > 32) return false;
    std::vector<int> map(np * hs, -1);
    for (int pi = 0; pi < hs; ++pi) {
        int last = -1;
        for (int o = 0; o < noff; ++o) {
            const int r = pi - nl.dh[o];
            if (((r % hs) + hs) % hs) continue;
            const int p = (int)(std::lower_bound(keys.begin(), keys.end(), std::make_pair(nl.dt[o], -(r / hs))) -
                                keys.begin());
            if (p <= last || map[p * hs + pi] >= 0) return false;  // the residue's tap order not kept
            map[p * hs + pi] = o;
            last = p;
        }
    }
    nl.wm = net->dalloc((size_t)np * hs * L.fin * L.fout * 2);
    if (!nl.wm) return false;
    nl.wm_map = map;
    nl.wm_dt.resize(np);
    nl.wm_dh.resize(np);
    for (int p = 0; p < np; ++p) {
        nl.wm_dt[p] = keys[p].first;
        nl.wm_dh[p] = -keys[p].second;
    }
    nl.wm_np = np;
    return true;
}
// conv input gradient with the weights as a plain [taps * fout x fin] B, N contiguous (the
// forward's B layout): block i = (tap taps[i]'s fin rows of W)^T, one batched transpose per
// layer and step. The shifted k-contiguous weight rows (op_wrows, the BROW halo kernels) ran
// cnn4's input gradient at half the forward's rate. KF_DGRAD_WT=0: op_wrows. The K order is
// the same either way, so the result is bit-identical.
static bool dgrad_wt_on() {
    const char *e = getenv("KF_DGRAD_WT");
    return !(e && e[0] == '0');
}
static void *dgrad_wt(KfNet *net, NetLayer &nl, const std::vector<int> &taps) {
    const Layer &L = nl.L;
    const size_t blk = (size_t)L.fin * L.fout * 2;
    if ((int)taps.size() > KF_TRANSPOSE_MAX || taps.size() > nl.dt.size()) return nullptr;
    if (!nl.wtd) nl.wtd = net->dalloc(nl.dt.size() * blk);
    if (!nl.wtd) return nullptr;
    std::vector<const void *> src;
    std::vector<void *> dst;
    std::vector<int> M, N;
    for (size_t i = 0; i < taps.size(); ++i) {
        src.push_back((const char *)wptr(net, nl.pW) + taps[i] * blk);
        dst.push_back((char *)nl.wtd + i * blk);
        M.push_back(L.fin);
        N.push_back(L.fout);
    }
    if (kf_transpose_batch((int)taps.size(), src.data(), dst.data(), M.data(), N.data()) != 0) return nullptr;
    return nl.wtd;
}
// compact row of source row t (nnet_set_row_subsampling), or -1 when t is not in the set
static inline int compact_of(const KfNet *net, int t) {
    const int T = net->T, nt = net->Tc - net->Tc0;
    if (t % 3 == 0 && t / 3 < net->Tc0) return t / 3;
    if (nt > 0 && t % 3 == (T - 1) % 3 && t >= T - 1 - 3 * (nt - 1) && t < T) return net->Tc - 1 - (T - 1 - t) / 3;
    return -1;
}
static const void *act_of(KfNet *net, int idx) {
    if (idx == -2) return net->ivec;
    if (idx < 0) return net->features;
    NetLayer &nl = net->layers[idx];
    return nl.act_alias ? act_of(net, nl.input) : nl.act;
}

// ---------------------------------------------------------------------------
// MXFP8 forward (configs[4] of BASELINE.json: "OCP-FP8 MFMA GEMM path")
// Every dense GEMM of TDNN-F / linear / prefinal / output layers runs on
// v_mfma_scale_f32_16x16x128_f8f6f4 when its input has an MXFP8 copy; the
// copies are written by the producing GEMM's epilogue (out8), the weights are
// quantised after every parameter change. Widths are padded to 128 (zero
// elements, zero scale bytes), so splice parts stay whole K-steps.
// ---------------------------------------------------------------------------
namespace {
inline int pad128(int x) { return (x + 127) / 128 * 128; }

bool mx_alloc(KfNet *net, Mx &m, size_t rows, int width) {
    m.ld = pad128(width);
    m.q = (uint8_t *)net->dalloc(rows * m.ld + 64);
    m.s = (uint8_t *)net->dalloc(rows * (m.ld / 32) + 64);
    if (!m.q || !m.s) return false;
    bridge_gpu_memset(m.q, 0, rows * m.ld + 64);
    bridge_gpu_memset(m.s, 0, rows * (m.ld / 32) + 64);
    return true;
}
// W [nparts*rows x N] fp16 -> Mx [N x nparts*pad128(rows)]: one quantisation job per part
// (run together by quantise_weights)
bool mx_weights(KfNet *net, Mx &m, int pi, int nparts, int rows, int N, bool alloc,
                std::vector<KfQuantJob> &jobs) {
    const int part = pad128(rows);
    if (alloc) {
        m.ld = nparts * part;
        m.q = (uint8_t *)net->dalloc((size_t)N * m.ld + 64);
        m.s = (uint8_t *)net->dalloc((size_t)N * (m.ld / 32) + 64);
        if (!m.q || !m.s) return false;
    }
    const uint16_t *W = (const uint16_t *)wptr(net, pi);
    for (int p = 0; p < nparts; ++p)
        jobs.push_back(KfQuantJob{W + (size_t)p * rows * N, N, N, rows, 1, m.q + p * part, m.ld, m.s + p * part / 32,
                                  m.ld / 32});
    return true;
}
// W2 [2*bn x dout] -> w8d [bn x 2*pad128(dout)]: row j holds W2 rows j and bn + j, each
// quantised in 32-element blocks along dout (the reduction of the affine input gradient)
bool mx_dgrad_weights(KfNet *net, NetLayer &nl, bool alloc, std::vector<KfQuantJob> &jobs) {
    const int bn = nl.L.bottleneck, dout = nl.L.out_dim, part = pad128(dout);
    Mx &m = nl.w8d;
    if (alloc) {
        m.ld = 2 * part;
        m.q = (uint8_t *)net->dalloc((size_t)bn * m.ld + 64);
        m.s = (uint8_t *)net->dalloc((size_t)bn * (m.ld / 32) + 64);
        if (!m.q || !m.s) return false;
    }
    const uint16_t *W2 = (const uint16_t *)wptr(net, nl.pW2);
    for (int p = 0; p < 2; ++p)
        jobs.push_back(KfQuantJob{W2 + (size_t)p * bn * dout, dout, bn, dout, 0, m.q + p * part, m.ld,
                                  m.s + p * part / 32, m.ld / 32});
    return true;
}
// the layer's output can carry an MXFP8 copy (its epilogue has 32-column blocks)
bool f8_producer(const KfNet *net, int idx) {
    const NetLayer &nl = net->layers[idx];
    const Layer &L = nl.L;
    // conv: the epilogue's [(t,h) x fout] view must be the consumer's [t x hout*fout], and
    // only a non-conv consumer reads the copy (a conv's input is the fp16 halo image)
    if (L.type == LayerType::ConvReluBN) {
        bool mx_consumer = false;
        for (const auto &c : net->layers)
            mx_consumer = mx_consumer || (c.input == idx && c.L.type != LayerType::ConvReluBN);
        return mx_consumer && L.fin != 1 && L.fout % 32 == 0 && L.out_dim % 128 == 0;
    }
    return L.type == LayerType::TDNNF || L.type == LayerType::Linear ||
           (L.type == LayerType::Prefinal && L.small_dim % 32 == 0);
}
// MXFP8 operand over an Mx tensor of T rows: plain, or spliced [x(t+dt0) | x(t+dt1)]
KfOperand op_mx(const Mx &m, int T, int nparts, int dt0, int dt1) {
    KfOperand o = op_base(m.q, m.ld, T, nparts * m.ld, 1);
    if (nparts == 2) {
        o.nparts = 2;
        o.part_width = m.ld;
        o.dt[0] = dt0;
        o.dt[1] = dt1;
        o.tpolicy = KF_CLAMP;
    }
    o.fmt = KF_FMT_MXFP8;
    o.scales = m.s;
    o.lds = m.ld / 32;
    return o;
}
KfOperand op_mxw(const Mx &m, int N) {
    KfOperand o = op_base(m.q, m.ld, N, m.ld, 1);
    o.fmt = KF_FMT_MXFP8;
    o.scales = m.s;
    o.lds = m.ld / 32;
    return o;
}
void set_out8(KfEpilogue &E, const Mx &m) {
    if (!m.q) return;
    E.out8 = m.q;
    E.ldo8 = m.ld;
    E.scale8 = m.s;
}
}  // namespace

// MXFP8 copy of a layer's input, or NULL (fp8 off / producer without one)
static const Mx *in8(KfNet *net, const NetLayer &nl) {
    if (!net->fp8 || nl.input < 0) return nullptr;
    const NetLayer &p = net->layers[nl.input];
    if (p.act_alias) return in8(net, p);
    return p.a8.q ? &p.a8 : nullptr;
}

static bool quantise_weights(KfNet *net, bool alloc) {
    std::vector<KfQuantJob> jobs;
    for (auto &nl : net->layers) {
        const Layer &L = nl.L;
        bool ok = true;
        switch (L.type) {
            case LayerType::TDNNF: {
                const int np = L.time_stride > 0 ? 2 : 1;
                ok = mx_weights(net, nl.w8, nl.pW, np, L.in_dim, L.bottleneck, alloc, jobs) &&
                     mx_weights(net, nl.w8b, nl.pW2, np, L.bottleneck, L.out_dim, alloc, jobs) &&
                     (np == 1 || mx_dgrad_weights(net, nl, alloc, jobs));
                break;
            }
            case LayerType::Linear:
            case LayerType::Output:
                ok = mx_weights(net, nl.w8, nl.pW, 1, L.in_dim, L.out_dim, alloc, jobs);
                break;
            case LayerType::Prefinal:
                ok = mx_weights(net, nl.w8, nl.pW, 1, L.in_dim, L.big_dim, alloc, jobs) &&
                     mx_weights(net, nl.w8b, nl.pW2, 1, L.big_dim, L.small_dim, alloc, jobs);
                break;
            default:
                break;
        }
        if (!ok) return false;
    }
    for (size_t j = 0; j < jobs.size(); j += KF_QUANT_MAX)
        if (!ck(kf_quant_mxfp8_batch((int)std::min<size_t>(KF_QUANT_MAX, jobs.size() - j), jobs.data() + j),
                "quantise weights"))
            return false;
    return true;
}

extern "C" int nnet_set_fp8(KfNet *net, int on) {
    kf_take_pending(__func__);
    if (!on_device(net, "set_fp8")) return -1;
    if (!on) {
        net->fp8 = 0;
        return 0;
    }
    net->fp8_dgrad = on != 2;
    if (!net->fp8) {
        const size_t T = (size_t)net->max_T;
        bool first = true;
        for (auto &nl : net->layers) first = first && !nl.w8.q;
        for (size_t i = 0; i < net->layers.size(); ++i) {
            NetLayer &nl = net->layers[i];
            const Layer &L = nl.L;
            if (first && f8_producer(net, (int)i) && !mx_alloc(net, nl.a8, T, L.out_dim)) {
                set_err("fp8: alloc " + L.name);
                return -1;
            }
            if (first && (L.type == LayerType::TDNNF || L.type == LayerType::Prefinal) &&
                !mx_alloc(net, nl.x8, T, L.type == LayerType::TDNNF ? L.bottleneck : L.big_dim)) {
                set_err("fp8: alloc " + L.name);
                return -1;
            }
        }
        // dz copies for the TDNN-F affine input gradients: as wide as the widest such layer
        int dzw = 0;
        for (auto &nl : net->layers)
            if (nl.L.type == LayerType::TDNNF && nl.L.time_stride > 0) dzw = std::max(dzw, nl.L.out_dim);
        for (int i = 0; first && dzw > 0 && i < 3; ++i)
            if (!mx_alloc(net, net->dz8[i], T, dzw)) {
                set_err("fp8: alloc dz copies");
                return -1;
            }
        if (!quantise_weights(net, first)) return -1;
    }
    net->fp8 = 1;
    return 0;
}

// ---------------------------------------------------------------------------
// forward (Network.Forward, forward.go:148-202)
// ---------------------------------------------------------------------------
static int forward_impl(KfNet *net, const void *features, int T);
extern "C" int nnet_forward(KfNet *net, const void *features, int T) {
    kf_take_pending(__func__);
    if (net->ivec_dim) {
        set_err("forward: the network has an ivector input; use nnet_forward_ivector");
        return -1;
    }
    return forward_impl(net, features, T);
}
// forward with per-sequence ivectors: ivectors fp16 [B x ivec_dim] on the device,
// seq_row0 host int[B+1] frame offsets (seq_row0[0] = 0, seq_row0[B] = T)
extern "C" int nnet_forward_ivector(KfNet *net, const void *features, int T, const void *ivectors, int B,
                                    const int *seq_row0) {
    kf_take_pending(__func__);
    if (!on_device(net, "forward_ivector")) return -1;
    // validate everything before touching the device or the network's state
    if (T <= 0 || T > net->max_T) {
        set_err("forward_ivector: T=" + std::to_string(T) + " outside (0, max_frames]");
        return -1;
    }
    if (!net->ivec_dim || !ivectors || B <= 0 || B > T || !seq_row0 || seq_row0[0] != 0 || seq_row0[B] != T) {
        set_err("forward_ivector: needs an ivector input layer, B in [1, T] and seq_row0[0] = 0, seq_row0[B] = T");
        return -1;
    }
    for (int s = 0; s < B; ++s)
        if (seq_row0[s + 1] <= seq_row0[s]) {
            set_err("forward_ivector: empty or unordered sequence " + std::to_string(s));
            return -1;
        }
    if (!net->seq_off) {
        net->seq_off = (int *)net->dalloc(((size_t)net->max_T + 1) * 4);
        if (!net->seq_off) {
            set_err("alloc seq offsets");
            return -1;
        }
    }
    if (bridge_transfer_int32(net->seq_off, seq_row0, (size_t)B + 1)) {
        set_err("upload seq offsets");
        return -1;
    }
    net->ivec = ivectors;
    net->B = B;
    return forward_impl(net, features, T);
}
// k-contiguous (transposed) copies of the short-K forward weights: the tiled GEMM's
// k-contiguous B path beats its reduction-major one on these shapes (TDNN-F affine
// forward with the full epilogue 243 -> 225 us, DESIGN.md §7 performance log, r2)
static bool refresh_wt(KfNet *net) {
    if (!net->wt_dirty) return true;
    // one launch for every layer's copy (was one ops_transpose each: 18 x 9 us per step)
    std::vector<const void *> src;
    std::vector<void *> dst;
    std::vector<int> M, N;
    auto flush = [&]() {
        const bool ok = src.empty() || ck(kf_transpose_batch((int)src.size(), src.data(), dst.data(), M.data(),
                                                             N.data()),
                                          "transpose weights");
        src.clear(), dst.clear(), M.clear(), N.clear();
        return ok;
    };
    for (auto &nl : net->layers) {
        if (!nl.wt) continue;
        src.push_back(wptr(net, nl.wt_pi));
        dst.push_back(nl.wt);
        M.push_back(nl.wt_K);
        N.push_back(nl.wt_N);
        if ((int)src.size() == KF_TRANSPOSE_MAX && !flush()) return false;
    }
    if (!flush()) return false;
    net->wt_dirty = false;
    return true;
}
static int forward_impl(KfNet *net, const void *features, int T) {
    if (!on_device(net, "forward")) return -1;
    if (!refresh_wt(net)) return -1;
    if (T <= 0 || T > net->max_T) {
        set_err("forward: T=" + std::to_string(T) + " outside (0, max_frames]");
        return -1;
    }
    net->T = T;
    net->features = features;
    net->Tc = net->Tc0 = 0;
    if (net->rsub && net->first_c >= 0 && !net->fp8 && !net->implicit_dz) {
        const int nt = (T - 1) % 3 == 0 ? 0 : net->rs_nt;
        const int tc0 = (T - 1) / 3 + 1;
        if (tc0 >= 4 * nt + 16 && tc0 + nt <= net->maxTc) {
            net->Tc0 = tc0;
            net->Tc = tc0 + nt;
        }
    }
    for (size_t li = 0; li < net->layers.size(); ++li) {
        NetLayer &nl = net->layers[li];
        const Layer &L = nl.L;
        const void *x = act_of(net, nl.input);
        if (net->Tc && (int)li == net->first_c && !net->conv_c) {  // the conv stack's output on the compact rows
            if (!ck(kf_gather_rows(net->xc, x, (long long)L.in_dim * 2, T, net->Tc0, net->Tc), "row set gather"))
                return -1;
            x = net->xc;
        }
        const int Tl = rows_of(net, (int)li);
        const int din = L.in_dim, dout = L.out_dim;
        switch (L.type) {
            case LayerType::IDCT:
                if (!ck(kf_small_gemm(x, din, nl.idct, nl.act, dout, T, din, dout), "idct")) return -1;
                break;
            case LayerType::Batchnorm:
                if (!ck(kf_bn_apply(x, nl.act, nl.per_seq ? net->B : T, dout, nl.bn_scale, nl.bn_shift),
                        "batchnorm"))
                    return -1;
                break;
            case LayerType::SpecAugment:
                break;  // pass-through (forward.go:225-231, masking is a TODO there too)
            case LayerType::CombineFeatureMaps:
                if (nl.input2 != -100) {  // Append(a, b): b broadcast per sequence when per_seq
                    const bool bseq = nl.input2 == -2 || (nl.input2 >= 0 && net->layers[nl.input2].per_seq);
                    if (!ck(kf_combine_feature_maps(x, L.height * L.nf1, act_of(net, nl.input2), L.height * L.nf2,
                                                    bseq ? net->seq_off : nullptr, net->B, nl.act, dout, T,
                                                    L.height, L.nf1, L.nf2),
                            "combine"))
                        return -1;
                } else if (!ck(ops_copy(nl.act, x, T * dout), "combine copy") ||
                           !ck(ops_combine_feature_maps(nl.act, T, dout, L.height, L.nf1, L.nf2), "combine")) {
                    return -1;
                }
                break;
            case LayerType::ConvReluBN: {
                if (L.fin == 1) {
                    if (!ck(kf_conv_c1_forward(T, L.hin, L.hout, L.hsub, L.fout, (int)nl.dt.size(),
                                               nl.dt.data(), nl.dh.data(), x, wptr(net, nl.pW),
                                               wptr(net, nl.pb), nl.bn_scale, nl.bn_shift, nl.act,
                                               nl.mask),
                            "conv c1"))
                        return -1;
                    break;
                }
                const int K = (int)nl.dt.size() * L.fin;
                if (nl.kp) {  // small fin (Kaldi's cnn1 after combine-feature-maps: 6): im2col + GEMM
                    if (!ck(kf_im2col_small(x, din, T, L.hin, L.hout, L.hsub, L.fin, (int)nl.dt.size(),
                                            nl.dt.data(), nl.dh.data(), nl.im2col, nl.kp),
                            "im2col small") ||
                        !ck(ops_copy(nl.wpad, wptr(net, nl.pW), K * L.fout), "conv weight pad"))
                        return -1;
                    KfOperand A = op_base(nl.im2col, nl.kp, T * L.hout, nl.kp, 1);
                    KfOperand B = op_base(nl.wpad, L.fout, nl.kp, L.fout, 0);
                    KfEpilogue E = epi0();
                    E.out = nl.act;
                    E.ldo = L.fout;
                    E.bias = wptr(net, nl.pb);
                    E.relu = 1;
                    E.mask_out = nl.mask;
                    E.scale = nl.bn_scale;
                    E.shift = nl.bn_shift;
                    if (!ck(kf_gemm_fused(T * L.hout, L.fout, nl.kp, &A, &B, &E), "conv small fin")) return -1;
                    break;
                }
                KfOperand A = op_im2col(nl, x, T, 1);
                KfOperand B = op_base(wptr(net, nl.pW), L.fout, K, L.fout, 0);
                KfEpilogue E = epi0();
                E.out = nl.act;
                E.ldo = L.fout;
                E.bias = wptr(net, nl.pb);
                E.relu = 1;
                E.mask_out = nl.mask;
                E.scale = nl.bn_scale;
                E.shift = nl.bn_shift;
                if (net->fp8 && nl.a8.q) {  // rows (t,h) of fout: the [t x hout*fout] copy
                    E.out8 = nl.a8.q;
                    E.ldo8 = L.fout;
                    E.scale8 = nl.a8.s;
                }
                if (conv_compact(net, (int)li)) {
                    // output frames 3c (c < Tc0), and the tail T-1-3(nt-1) ... T-1 (compact rows
                    // Tc0 ..): two time-strided launches into compact rows. The tail's few
                    // workgroups (latency: the whole K loop for ~200 rows) run beside the main
                    // launch on the weight-gradient stream.
                    const int nt = net->Tc - net->Tc0;
                    void *const cst = kf_get_stream();
                    const bool side = nt > 0 && net->wg_stream;
                    if (nt > 0) {
                        const size_t r0 = (size_t)net->Tc0 * L.hout * L.fout;  // elements
                        KfOperand At = A;
                        At.tmul = 3;
                        At.t0 = T - 1 - 3 * (nt - 1);
                        At.nrows = nt * L.hout;
                        KfEpilogue Et = E;
                        Et.out = (char *)nl.act + r0 * 2;
                        Et.mask_out = nl.mask + r0 / 8;
                        if (side && (kf_event_record(net->ev_go, cst) != 0 || kf_stream_wait(net->wg_stream, net->ev_go) != 0)) {
                            set_err("forward: conv tail stream order");
                            return -1;
                        }
                        if (side) kf_set_stream(net->wg_stream);
                        const bool ok = ck(kf_gemm_fused(nt * L.hout, L.fout, K, &At, &B, &Et), "conv (compact tail rows)");
                        const bool rec = !side || kf_event_record(net->ev_aux, net->wg_stream) == 0;
                        kf_set_stream(cst);
                        if (!ok) return -1;
                        if (!rec) {
                            set_err("forward: conv tail event");
                            return -1;
                        }
                    }
                    A.tmul = 3;
                    A.nrows = net->Tc0 * L.hout;
                    if (!ck(kf_gemm_fused(net->Tc0 * L.hout, L.fout, K, &A, &B, &E), "conv (compact rows)"))
                        return -1;
                    if (side && kf_stream_wait(cst, net->ev_aux) != 0) {
                        set_err("forward: conv tail join");
                        return -1;
                    }
                    break;
                }
                if (!ck(kf_gemm_fused(T * L.hout, L.fout, K, &A, &B, &E), "conv")) return -1;
                break;
            }
            case LayerType::TDNNF: {
                const int T = Tl;  // compact rows (rows_of)
                const int s = nl.compact && net->Tc ? L.time_stride / 3 : L.time_stride, bn = L.bottleneck;
                const int klin = s > 0 ? 2 * din : din, kaff = s > 0 ? 2 * bn : bn;
                const int np = s > 0 ? 2 : 1;
                const Mx *x8 = in8(net, nl);
                KfOperand A = x8 ? op_mx(*x8, T, np, -s, 0)
                                 : s > 0 ? op_splice(x, T, din, -s, 0, KF_CLAMP, 1) : op_base(x, din, T, din, 1);
                // compact rows with a tail: row Tc0 - 1's +1 neighbour in the affine splice is row
                // T-1 (the tail's last row). The scratch row Tc0 reads the last row's linear inputs
                // [x(Tc-1-s) | x(Tc-1)] (edge rows), so its bottleneck is that row's, bit for bit
                // (nnet_set_row_subsampling)
                const bool scratch = nl.compact && net->Tc > net->Tc0 && s > 0;
                if (scratch && !x8) {
                    A.edge_t[0] = A.edge_t[1] = net->Tc0;
                    A.edge_row[0] = std::max(0, net->Tc - 1 - s);
                    A.edge_row[1] = net->Tc - 1;
                }
                KfOperand B = x8 ? op_mxw(nl.w8, bn) : op_base(wptr(net, nl.pW), bn, klin, bn, 0);
                KfEpilogue E = epi0();
                E.out = nl.aux;
                E.ldo = bn;
                // the bottleneck's MXFP8 copy is quantised after the GEMM rather than in its
                // epilogue: out8 needs 32-column blocks inside one wave's tile, which would
                // force 256x256 tiles onto N = bottleneck (320 of 512 columns used) instead of
                // 384x160 (3072 model: 331 -> see DESIGN §7)
                if (!ck(kf_gemm_fused(T, bn, x8 ? nl.w8.ld : klin, &A, &B, &E), "tdnnf linear")) return -1;
                if (scratch && x8 &&
                    !ck(ops_copy((char *)nl.aux + (size_t)net->Tc0 * bn * 2,
                                 (const char *)nl.aux + (size_t)(net->Tc - 1) * bn * 2, bn),
                        "row set edge copy"))
                    return -1;
                if (net->fp8 && nl.x8.q &&
                    !ck(kf_quant_mxfp8(nl.aux, bn, T, bn, 0, nl.x8.q, nl.x8.ld, nl.x8.s, nl.x8.ld / 32),
                        "quantise bottleneck"))
                    return -1;
                const bool f8b = net->fp8 && nl.x8.q;
                KfOperand A2 = f8b ? op_mx(nl.x8, T, np, 0, s)
                                   : s > 0 ? op_splice(nl.aux, T, bn, 0, s, KF_CLAMP, 1)
                                           : op_base(nl.aux, bn, T, bn, 1);
                KfOperand B2 = f8b             ? op_mxw(nl.w8b, dout)
                       : nl.wt               ? op_base(nl.wt, kaff, dout, kaff, 1)
                                             : op_base(wptr(net, nl.pW2), dout, kaff, dout, 0);
                KfEpilogue E2 = epi0();
                if (net->fp8) set_out8(E2, nl.a8);
                E2.out = nl.act;
                E2.ldo = dout;
                E2.bias = wptr(net, nl.pb2);
                E2.relu = 1;
                E2.mask_out = nl.mask;
                E2.scale = nl.bn_scale;
                E2.shift = nl.bn_shift;
                if (nl.bypass) {
                    E2.resid = x;
                    E2.ldr = din;
                    E2.resid_alpha = (float)L.bypass_scale;
                }
                if (!ck(kf_gemm_fused(T, dout, f8b ? nl.w8b.ld : kaff, &A2, &B2, &E2), "tdnnf affine"))
                    return -1;
                break;
            }
            case LayerType::Linear: {
                const int T = Tl;
                if (nl.per_seq) {  // ReplaceIndex branch: one row per sequence, any dims (ivector 100)
                    if (!ck(kf_rows_gemm(x, din, wptr(net, nl.pW), dout, nl.act, dout, net->B, din, dout),
                            "ivector linear"))
                        return -1;
                    break;
                }
                const Mx *x8 = in8(net, nl);
                KfOperand A = x8 ? op_mx(*x8, T, 1, 0, 0) : op_base(x, din, T, din, 1);
                KfOperand B = x8 ? op_mxw(nl.w8, dout) : op_base(wptr(net, nl.pW), dout, din, dout, 0);
                KfEpilogue E = epi0();
                E.out = nl.act;
                E.ldo = dout;
                if (net->fp8) set_out8(E, nl.a8);
                if (!ck(kf_gemm_fused(T, dout, x8 ? nl.w8.ld : din, &A, &B, &E), "linear")) return -1;
                break;
            }
            case LayerType::Attention: {
                // affine on the GPU (forward.go:813-826), then the per-head attention with
                // ReLU + BatchNorm fused (the reference's CPU loop, :850-908)
                const int A = att_affine(L);
                KfOperand Aop = op_base(x, din, T, din, 1);
                KfOperand B = op_base(wptr(net, nl.pW), A, din, A, 0);
                KfEpilogue E = epi0();
                E.out = nl.aux;
                E.ldo = A;
                E.bias = wptr(net, nl.pb);
                if (!ck(kf_gemm_fused(T, A, din, &Aop, &B, &E), "attention affine")) return -1;
                KfAttention att = att_args(nl, T);
                if (!ck(kf_attention_forward(&att, nl.act, dout, nl.mask, nl.bn_scale, nl.bn_shift), "attention"))
                    return -1;
                break;
            }
            case LayerType::Prefinal: {
                const int T = Tl;
                const int big = L.big_dim, small = L.small_dim;
                const Mx *x8 = in8(net, nl);
                KfOperand A = x8 ? op_mx(*x8, T, 1, 0, 0) : op_base(x, din, T, din, 1);
                KfOperand B = x8                    ? op_mxw(nl.w8, big)
                              : nl.wt               ? op_base(nl.wt, din, big, din, 1)
                                                    : op_base(wptr(net, nl.pW), big, din, big, 0);
                KfEpilogue E = epi0();
                if (net->fp8) set_out8(E, nl.x8);
                E.out = nl.aux;
                E.ldo = big;
                E.bias = wptr(net, nl.pb);
                E.relu = 1;
                E.mask_out = nl.mask;
                E.scale = nl.bn_scale;
                E.shift = nl.bn_shift;
                if (!ck(kf_gemm_fused(T, big, x8 ? nl.w8.ld : din, &A, &B, &E), "prefinal big")) return -1;
                const bool f8b = net->fp8 && nl.x8.q;
                KfOperand A2 = f8b ? op_mx(nl.x8, T, 1, 0, 0) : op_base(nl.aux, big, T, big, 1);
                KfOperand B2 = f8b ? op_mxw(nl.w8b, small) : op_base(wptr(net, nl.pW2), small, big, small, 0);
                KfEpilogue E2 = epi0();
                if (net->fp8) set_out8(E2, nl.a8);
                E2.out = nl.act;
                E2.ldo = small;
                if (nl.has_bn2) {
                    E2.scale = nl.bn2_scale;
                    E2.shift = nl.bn2_shift;
                }
                if (!ck(kf_gemm_fused(T, small, f8b ? nl.w8b.ld : big, &A2, &B2, &E2), "prefinal small"))
                    return -1;
                break;
            }
            case LayerType::Output: {
                const int T = Tl;
                const Mx *x8 = in8(net, nl);
                KfOperand A = x8 ? op_mx(*x8, T, 1, 0, 0) : op_base(x, din, T, din, 1);
                KfOperand B = x8 ? op_mxw(nl.w8, dout) : op_base(wptr(net, nl.pW), dout, din, dout, 0);
                KfEpilogue E = epi0();
                E.out = nl.act;
                E.ldo = dout;
                E.bias = wptr(net, nl.pb);
                if (!ck(kf_gemm_fused(T, dout, x8 ? nl.w8.ld : din, &A, &B, &E), "output")) return -1;
                if (L.include_log_softmax && !ck(ops_log_softmax(nl.act, T, dout), "log_softmax"))
                    return -1;
                break;
            }
            default:
                set_err("forward: unsupported layer " + L.name);
                return -1;
        }
    }
    return 0;
}

extern "C" const void *nnet_activation(const KfNet *cnet, const char *layer, int *rows, int *cols) {
    KfNet *net = const_cast<KfNet *>(cnet);
    for (size_t i = 0; i < net->layers.size(); ++i)
        if (net->layers[i].L.name == layer) {
            if (rows) *rows = act_rows(net, (int)i);  // compact rows above the conv stack (row subsampling)
            if (cols) *cols = net->layers[i].L.out_dim;
            return act_of(net, (int)i);
        }
    set_err(std::string("no layer ") + layer);
    return nullptr;
}

// ---------------------------------------------------------------------------
// backward (Network.Backward, network_backward.go:94-143) — exact gradients
// ---------------------------------------------------------------------------
namespace {

// ring index of an input-gradient buffer, or -1
int dz_index(const KfNet *net, const void *p) {
    for (int i = 0; i < 3; ++i)
        if (p == net->dz[i]) return i;
    return -1;
}

// Epilogue of an input-gradient GEMM that produces the gradient of layer P
// (the input of the layer being back-propagated). v = acc (+ bypass * g_cur):
//   g_P = rne(v) when P itself has a bypass (its own input gradient needs it)
//   dz_P = rne(v * bnscale_P * mask_P) for relu+BN layers, rne(v*bn2scale) for prefinal
bool dx_epilogue(KfNet *net, int P, void *dz_out, void *g_out, KfEpilogue &E) {
    E = epi0();
    NetLayer &pl = net->layers[P];
    const Layer &L = pl.L;
    const int w = L.out_dim;
    E.ldo2 = w;
    E.out2 = dz_out;
    const int di = dz_index(net, dz_out);
    if (di >= 0) net->dz_imp[di] = net->dz_edge[di] = false;
    switch (L.type) {
        case LayerType::TDNNF: {
            E.scale2 = pl.bn_scale;
            E.mask_in = pl.mask;
            if (pl.bypass) {
                E.out = g_out;
                E.ldo = w;
                // implicit dz: g is stored anyway, its consumers apply mask and scale (the
                // masked weight gradient needs 256-column tiles: w > 128, not 160 / 320)
                const bool shape_ok = w > 128 && !(w % 160 == 0 && w <= 320);
                if (net->implicit_dz && !net->fp8 && di >= 0 && pl.mask && pl.bn_scale && net->w2s && shape_ok) {
                    E.out2 = nullptr;
                    E.scale2 = nullptr;
                    E.mask_in = nullptr;
                    net->dz_imp[di] = true;
                    return true;
                }
            }
            // a strided P's clamped-splice edge row (row T of dz: sum of its rows T-1-s .. T-1),
            // summed by the epilogue's last row tile instead of a separate kf_rows_sum launch
            if (L.time_stride > 0 && di >= 0 && net->T > 0 && !(net->Tc && pl.compact)) {
                const int T = net->T;
                E.edge_out = (char *)dz_out + (size_t)T * w * 2;
                E.edge_r0 = T - 1 - L.time_stride < 0 ? 0 : T - 1 - L.time_stride;
                E.edge_r1 = T;
                E.edge_src = 1;
                net->dz_edge[di] = true;
            }
            // MXFP8 train step: also the e4m3 copy of dz_P for P's affine input gradient; only
            // when the copy's row is exactly w wide (w % 128 == 0), so the dgrad GEMM's K range
            // holds no stale codes from a wider layer's copy
            const int i = dz_index(net, dz_out);
            if (net->fp8 && net->fp8_dgrad && i >= 0 && w % 128 == 0 && pl.w8d.q && net->dz8[i].q &&
                net->dz8[i].ld == w) {
                E.out8 = net->dz8[i].q;
                E.ldo8 = net->dz8[i].ld;
                E.scale8 = net->dz8[i].s;
                E.out8_src = 1;
                net->dz8_layer[i] = P;
            }
            return true;
        }
        case LayerType::ConvReluBN:
        case LayerType::Attention:
            E.scale2 = pl.bn_scale;
            E.mask_in = pl.mask;
            return true;
        case LayerType::Prefinal:
            if (pl.has_bn2) E.scale2 = pl.bn2_scale;
            return true;
        case LayerType::Batchnorm:
            // batchnorm-component (frozen statistics): the gradient at its input is the
            // output gradient times its per-column scale (backward_wrappers.cu:105-115),
            // applied in the producing GEMM's epilogue; the step through the BN layer is
            // then a pass-through (backward_impl). Its own input must take a raw gradient.
            if (pl.input < 0 || !(net->layers[pl.input].L.type == LayerType::Linear)) {
                set_err("backward: gradient through batchnorm-component " + L.name +
                        " into a layer other than linear-component is not supported");
                return false;
            }
            E.scale2 = pl.bn_scale;
            return true;
        case LayerType::Linear:
        case LayerType::CombineFeatureMaps:  // raw gradient; its backward splits it (ivector branch)
            return true;
        default:
            set_err("backward: gradient into layer " + L.name + " is not supported");
            return false;
    }
}

}  // namespace

static int backward_impl(KfNet *net, const void *out_grad, int max_layers);
static bool dp_issue(KfNet *net, size_t &next, int step);
extern "C" int nnet_backward(KfNet *net, const void *out_grad) {
    kf_take_pending(__func__);
    return backward_impl(net, out_grad, 1 << 30);
}
// debugging / tests: back-propagate through the top `n` layers only
extern "C" int nnet_backward_n(KfNet *net, const void *out_grad, int n) {
    return backward_impl(net, out_grad, n);
}
// debugging / tests: device pointers of internal tensors
extern "C" const void *nnet_debug_tensor(KfNet *net, const char *what, int layer) {
    std::string w = what;
    if (w == "dzlast") return net->dz_last;
    if (w == "dz0") return net->dz[0];
    if (w == "dz1") return net->dz[1];
    if (w == "dz2") return net->dz[2];
    if (w == "g2") return net->g[2];
    if (w == "g0") return net->g[0];
    if (w == "g1") return net->g[1];
    if (w == "dbott") return net->dbott_last ? net->dbott_last : net->dbott;
    // the MXFP8 copies of dz[layer] (layer = buffer 0 / 1) and the layer whose affine input
    // gradient reads it (as an int, through the pointer's low bits: -1 none), MXFP8 train step
    if ((w == "dz8q" || w == "dz8s" || w == "dz8layer") && layer >= 0 && layer <= 2) {
        if (w == "dz8layer") return (const void *)(intptr_t)(net->dz8_layer[layer] + 1);
        return w == "dz8q" ? (const void *)net->dz8[layer].q : (const void *)net->dz8[layer].s;
    }
    if (layer < 0 || layer >= (int)net->layers.size()) return nullptr;
    if (w == "aux") return net->layers[layer].aux;
    if (w == "dproj") return net->layers[layer].dproj;
    if (w == "mask") return net->layers[layer].mask;
    if (w == "bn_scale") return net->layers[layer].bn_scale;
    if (w == "bn2_scale") return net->layers[layer].bn2_scale;
    // the e4m3 affine weight rows of the MXFP8 input gradient, [bn x 2*pad128(out)]
    if (w == "w8dq") return net->layers[layer].w8d.q;
    if (w == "w8ds") return net->layers[layer].w8d.s;
    // the MXFP8 copy this layer's GEMM reads (e4m3 [T x pad128(in)], E8M0 [T x pad128(in)/32])
    if (w == "x8q" || w == "x8s") {
        const Mx *m = in8(net, net->layers[layer]);
        return !m ? nullptr : w == "x8q" ? (const void *)m->q : (const void *)m->s;
    }
    return nullptr;
}
static int backward_impl(KfNet *net, const void *out_grad, int max_layers) {
    if (!on_device(net, "backward")) return -1;
    const int T = net->T;
    if (T <= 0) {
        set_err("backward before forward");
        return -1;
    }
    const int n = (int)net->layers.size();
    // Two streams: the input-gradient chain on the caller's stream (main), every write into
    // the gradient buffer on the weight-gradient stream (side), which waits for main at each
    // wgrad(): the dW GEMMs of a layer overlap the input gradients below it. Hazards (WAR on
    // shared scratch) are ordered by events: the dz / g / dbott buffers cycle three deep and
    // main waits for a step's side work before it overwrites what that work read (dx_wait,
    // side_wait). All gradient writes (and so the data-parallel
    // bucket gates, dp_issue) are on side; main joins side before returning.
    void *const caller = kf_get_stream();
    void *mainst = caller;
    const bool two = net->wg_side != 0 && net->wg_stream != nullptr;
    struct Restore {  // every return leaves the caller's stream current
        void *s;
        ~Restore() { kf_set_stream(s); }
    } restore{caller};
    // With the weight-gradient stream the input-gradient chain runs on a high-priority
    // stream (its workgroups are dispatched ahead of the weight gradients') and each weight
    // gradient launches 256 workgroups instead of 512. Same-box A/B (bench default, 20
    // steps, median): one stream 38.13 / 38.36 ms, two streams 37.57 / 37.52;
    // the chain's priority is neutral (37.55 without it), 512-workgroup weight gradients
    // cost 1.2 ms (38.78). With the row-subsampled step (r6) 160 workgroups: non-den step
    // time 17.52 ms against 17.81 at 256, 17.57 at 128, 18.15 at 96 (same box, 3 runs each).
    // (A/B knobs: KF_BWD_HP=0 keeps the chain on the caller's stream, KF_BWD_WGT=<n> sets
    // the weight gradients' workgroup target)
    static const int env_hp = getenv("KF_BWD_HP") ? atoi(getenv("KF_BWD_HP")) : 1;
    static const int env_wgt = getenv("KF_BWD_WGT") ? atoi(getenv("KF_BWD_WGT")) : 160;
    const bool hp = two && net->hp_stream && env_hp;
    struct Target {
        int old;
        ~Target() { kf_gemm_wgrad_target(old); }
    } target{kf_gemm_wgrad_target(two ? env_wgt : 0)};
    if (hp) {
        if (kf_event_record(net->ev_go, caller) != 0 || kf_stream_wait(net->hp_stream, net->ev_go) != 0) {
            set_err("backward: chain stream order");
            return -1;
        }
        mainst = net->hp_stream;
        kf_set_stream(mainst);
    }
    auto to_side = [&]() -> bool {  // side continues after everything main enqueued so far
        if (!two) return true;
        if (kf_event_record(net->ev_go, mainst) != 0 || kf_stream_wait(net->wg_stream, net->ev_go) != 0) {
            set_err("backward: weight-gradient stream order");
            return false;
        }
        kf_set_stream(net->wg_stream);
        if (net->stall_side > 0 && kf_debug_spin(net->wg_stream, net->stall_side) != 0) {
            set_err("backward: debug stall");
            return false;
        }
        return true;
    };
    auto to_main = [&]() { kf_set_stream(mainst); };
    // Steps (layers that hand a gradient down) cycle through three dz / g / dbott buffers.
    // Before step i rewrites its dz / g buffers, main waits for the side work of step i - 2,
    // the last reader of what step i - 3 wrote there; before it rewrites its dbott buffer
    // (earlier in the step), for that of step i - 3. Step i - 1's side work keeps running.
    // The side stream is in order, so waiting for step j's event covers every step <= j.
    int stepi = 0, waited = -1;  // side work of steps <= waited: main has waited for it
    auto side_wait = [&](int upto) -> bool {
        if (!two || upto <= waited || upto < 0) return true;
        if (kf_stream_wait(mainst, net->ev_step[upto % 3]) != 0) {
            set_err("backward: weight-gradient stream join");
            return false;
        }
        waited = upto;
        return true;
    };
    auto dx_wait = [&]() -> bool { return side_wait(stepi - 2); };
    auto joined = [&]() { waited = stepi - 1; };
    // the top layer must be the chain output
    const void *dz = out_grad;  // gradient w.r.t. pre-activation of the current layer
    const void *gcur = out_grad;  // stored gradient w.r.t. the current layer's output
    int flip = 0, done = 0;
    // dbott cycles by TDNN-F / prefinal step (the steps that write it), not by layer: a
    // pass-through step in between (Batchnorm) must not advance it, or the next step would
    // reuse a buffer whose weight gradient may still read it (side_wait covers step i - 3).
    int nbott = 0;
    size_t dp_next = 0;
    if (!to_side()) return -1;
    for (const auto &r : net->offpath) bridge_gpu_memset(net->grad + r.first, 0, (size_t)r.second * 4);
    (void)n;
    // negative control of the data-parallel tests: exchanging before any producer ran
    if (net->dp && net->dp_early) {
        if (!dp_issue(net, dp_next, INT_MAX)) return -1;
        // ... and finished before any producer writes (deterministic: left to race with the
        // backward, a fast one could finish first and hide the early exchange)
        if (kf_dp_join(net->dp) != 0 ||
            (two && (kf_event_record(net->ev_side, net->wg_stream) != 0 || kf_stream_wait(mainst, net->ev_side) != 0))) {
            set_err("backward: early-exchange join");
            return -1;
        }
    }
    to_main();
    // the bottleneck-gradient row mask of this row set (rebuilt when the set changes, on the
    // chain stream, which reads it): every 3-strided compact TDNN-F layer of one bottleneck
    // width zeroes the scratch row through it
    if (net->Tc > net->Tc0 && net->rowmask) {
        int bn = 0;
        for (size_t li = net->first_c; li < net->layers.size(); ++li) {
            const Layer &q = net->layers[li].L;
            if (q.type != LayerType::TDNNF || q.time_stride == 0) continue;
            bn = bn == 0 || bn == q.bottleneck ? q.bottleneck : -1;
        }
        if (bn > 0 && bn % 8 == 0 && (net->rm_bn != bn || net->rm_tc0 != net->Tc0 || net->rm_tc != net->Tc)) {
            bridge_gpu_memset(net->rowmask, 0xFF, (size_t)net->Tc * bn / 8);
            bridge_gpu_memset(net->rowmask + (size_t)net->Tc0 * bn / 8, 0, (size_t)bn / 8);
            net->rm_bn = bn;
            net->rm_tc0 = net->Tc0;
            net->rm_tc = net->Tc;
        }
    }
    const int Tfull = T;
    for (int li = net->chain_out; li >= 0 && done < max_layers; li = net->layers[li].input, ++done) {
        NetLayer &nl = net->layers[li];
        const Layer &L = nl.L;
        const int T = rows_of(net, li);  // compact rows above the conv stack (row subsampling)
        // the first compact layer's input gradient: in compact rows with the input layer's
        // mask gathered to them, then scattered to the full rows below (zero elsewhere)
        const bool to_full = net->Tc && li == net->first_c;
        const int din = L.in_dim, dout = L.out_dim;
        // (the first compact layer read its input gathered to the compact rows)
        const void *x = net->Tc && li == net->first_c && !net->conv_c ? net->xc : act_of(net, nl.input);
        bool want_dx = nl.needs_dx && nl.input >= 0;
        void *dz_next = net->dz[flip], *g_next = net->g[flip];
        // (this step's dbott buffer was last written at step i - 3 or earlier)
        void *const dbott_buf = !two ? net->dbott : nbott % 3 == 0 ? net->dbott : nbott % 3 == 1 ? net->dbott2 : net->dbott3;
        if (!side_wait(stepi - 3)) return -1;
        net->dz8_layer[flip] = -1;
        KfEpilogue E;
        if (want_dx && !dx_epilogue(net, nl.input, dz_next, g_next, E)) return -1;
        if (want_dx && to_full) {
            const NetLayer &pl = net->layers[nl.input];
            const int w = pl.L.out_dim;
            if (E.out || !E.out2 || E.edge_out || E.out8 || (E.mask_in && !pl.mask) || (w * 2) % 16 || (w / 8) % 16) {
                set_err("row subsampling: unsupported input gradient into " + pl.L.name);
                return -1;
            }
            if (E.mask_in && !net->conv_c) {  // (a compact conv's mask already is in compact rows)
                if (!ck(kf_gather_rows(net->mc, pl.mask, w / 8, Tfull, net->Tc0, net->Tc), "row set mask gather"))
                    return -1;
                E.mask_in = net->mc;
            }
            E.out2 = net->dzc;
        }
        // a weight gradient: on side, after what main enqueued so far
        auto wgrad = [&](const std::function<bool()> &f) -> bool {
            if (!to_side()) return false;
            const bool ok = f();
            to_main();
            return ok;
        };
        if (nl.bypass) {
            E.resid = gcur;
            E.ldr = dout;
            E.resid_alpha = (float)L.bypass_scale;
        }
        switch (L.type) {
            case LayerType::Output:
            case LayerType::Linear: {
                KfOperand A = op_base(x, din, T, din, 0);
                KfOperand B = op_base(dz, dout, T, dout, 0);
                if (!wgrad([&] {
                        return ck(kf_gemm_wgrad(din, dout, T, &A, &B, gptr(net, nl.pW), dout, gptr(net, nl.pb), 0),
                                  "wgrad");
                    }))
                    return -1;
                if (want_dx) {
                    KfOperand A2 = op_base(dz, dout, T, dout, 1);
                    KfOperand B2 = op_base(wptr(net, nl.pW), dout, din, dout, 1);
                    if (!dx_wait() || !ck(kf_gemm_fused(T, din, dout, &A2, &B2, &E), "dgrad")) return -1;
                }
                break;
            }
            case LayerType::Attention: {
                // dz = gradient at the attention output (pre-ReLU, from dx_epilogue);
                // exact attention backward into d(affine output), then the affine's
                // weight / bias / input gradients
                const int A = att_affine(L);
                KfAttention att = att_args(nl, T);
                if (!ck(kf_attention_backward(&att, dz, dout, nl.dproj, nl.att_scratch), "attention backward"))
                    return -1;
                KfOperand Aw = op_base(x, din, T, din, 0);
                KfOperand Bw = op_base(nl.dproj, A, T, A, 0);
                if (!wgrad([&] {
                        return ck(kf_gemm_wgrad(din, A, T, &Aw, &Bw, gptr(net, nl.pW), A, gptr(net, nl.pb), 0),
                                  "attention wgrad");
                    }))
                    return -1;
                if (want_dx) {
                    KfOperand A2 = op_base(nl.dproj, A, T, A, 1);
                    KfOperand B2 = op_base(wptr(net, nl.pW), A, din, A, 1);
                    if (!dx_wait() || !ck(kf_gemm_fused(T, din, A, &A2, &B2, &E), "attention dgrad")) return -1;
                }
                break;
            }
            case LayerType::Prefinal: {
                const int big = L.big_dim, small = L.small_dim;
                // dz = gradient at the small (BN2) pre-activation
                KfOperand A = op_base(nl.aux, big, T, big, 0);
                KfOperand B = op_base(dz, small, T, small, 0);
                if (!wgrad([&] {
                        return ck(kf_gemm_wgrad(big, small, T, &A, &B, gptr(net, nl.pW2), small, nullptr, 0),
                                  "prefinal small wgrad");
                    }))
                    return -1;
                void *dzbig = dbott_buf;
                net->dbott_last = dzbig;
                ++nbott;
                KfEpilogue E1 = epi0();
                E1.out2 = dzbig;
                E1.ldo2 = big;
                E1.scale2 = nl.bn_scale;
                E1.mask_in = nl.mask;
                KfOperand A1 = op_base(dz, small, T, small, 1);
                KfOperand B1 = op_base(wptr(net, nl.pW2), small, big, small, 1);
                if (!ck(kf_gemm_fused(T, big, small, &A1, &B1, &E1), "prefinal small dgrad")) return -1;
                KfOperand A3 = op_base(x, din, T, din, 0);
                KfOperand B3 = op_base(dzbig, big, T, big, 0);
                if (!wgrad([&] {
                        return ck(kf_gemm_wgrad(din, big, T, &A3, &B3, gptr(net, nl.pW), big, gptr(net, nl.pb), 0),
                                  "prefinal big wgrad");
                    }))
                    return -1;
                if (want_dx) {
                    KfOperand A4 = op_base(dzbig, big, T, big, 1);
                    KfOperand B4 = op_base(wptr(net, nl.pW), big, din, big, 1);
                    if (!dx_wait() || !ck(kf_gemm_fused(T, din, big, &A4, &B4, &E), "prefinal big dgrad")) return -1;
                }
                break;
            }
            case LayerType::TDNNF: {
                const int s = nl.compact && net->Tc ? L.time_stride / 3 : L.time_stride, bn = L.bottleneck;
                const int klin = s > 0 ? 2 * din : din, kaff = s > 0 ? 2 * bn : bn;
                // implicit dz (dx_epilogue): the layer's g read through its ReLU mask, the BN
                // scale applied to the weight gradient's columns and folded into W2 below
                const int ib = dz_index(net, dz);
                const bool imp = ib >= 0 && net->dz_imp[ib];
                const void *dzs = imp ? gcur : dz;
                auto masked = [&](KfOperand o) {
                    if (imp) {
                        o.mask = nl.mask;
                        o.mask_rows = T;
                    }
                    return o;
                };
                // affine weight / bias gradient: splice+(bott)^T . dz
                KfOperand A = s > 0 ? op_splice(nl.aux, T, bn, 0, s, KF_CLAMP, 0)
                                    : op_base(nl.aux, bn, T, bn, 0);
                KfOperand B = masked(op_base(dzs, dout, T, dout, 0));
                auto aff_wgrad = [&] {
                    if (imp)
                        return ck(kf_gemm_wgrad_scaled(kaff, dout, T, &A, &B, gptr(net, nl.pW2), dout,
                                                       gptr(net, nl.pb2), 0, nl.bn_scale),
                                  "tdnnf affine wgrad");
                    return ck(kf_gemm_wgrad(kaff, dout, T, &A, &B, gptr(net, nl.pW2), dout, gptr(net, nl.pb2), 0),
                              "tdnnf affine wgrad");
                };
                // The affine weight gradients run on the weight-gradient stream. (r5, with a
                // two-deep gradient ring, every other one ran on the chain: the chain waited for
                // the side stream before each linear input gradient, and that balanced the two,
                // 36.66 / 36.89 -> 36.55 / 36.65 ms. With the three-deep ring, all on side: 24.81 /
                // 24.89 against 24.96 / 25.13 ms every other, 25.51 / 25.69 all on the chain.)
                // KF_BWD_MAIN_AFF: 1 = every other on the chain, 2 = all on the chain (A/B).
                static const int env_main_aff = getenv("KF_BWD_MAIN_AFF") ? atoi(getenv("KF_BWD_MAIN_AFF")) : 0;
                const int main_aff = net->main_aff >= 0 ? net->main_aff : env_main_aff;
                const bool aff_on_main = two && (main_aff == 2 || (main_aff == 1 && (done & 1)));
                if (!aff_on_main && !wgrad(aff_wgrad)) return -1;
                const void *w2 = wptr(net, nl.pW2);
                if (imp) {
                    if (!ck(kf_scale_cols(w2, dout, nl.bn_scale, net->w2s, dout, kaff, dout), "tdnnf scaled W2")) return -1;
                    w2 = net->w2s;
                }
                // bottleneck gradient: transpose of the [0, +s] clamped splice
                void *dbott = dbott_buf;
                net->dbott_last = dbott;
                ++nbott;
                KfEpilogue E1 = epi0();
                E1.out = dbott;
                E1.ldo = bn;
                // compact rows with a tail: the scratch row Tc0 read row Tc0 - 1's gradient
                // through the +1 adjacency; its true gradient is zero (written as zero through
                // the row mask)
                bool zero_scratch = nl.compact && net->Tc > net->Tc0 && s > 0;
                if (zero_scratch && net->rowmask && net->rm_bn == bn && net->rm_tc0 == net->Tc0 &&
                    net->rm_tc == net->Tc) {
                    E1.out = nullptr;
                    E1.out2 = dbott;
                    E1.ldo2 = bn;
                    E1.mask_in = net->rowmask;
                    zero_scratch = false;
                }
                if (s > 0 && want_dx) {
                    // the linear input gradient's edge row (row T of dbott: sum of rows 0 .. s),
                    // summed by this GEMM's first row tile
                    E1.edge_out = (char *)dbott + (size_t)T * bn * 2;
                    E1.edge_r0 = 0;
                    E1.edge_r1 = s + 1 < T ? s + 1 : T;
                    E1.edge_src = E1.out2 ? 1 : 0;
                }
                const int i8 = dz_index(net, dz);
                if (s > 0) {
                    // spare row T of dz (of g when dz is implicit: the masked sum) holds
                    // sum_{t >= T-1-s} dz[t] (clamped-splice transpose)
                    void *edge = (char *)dzs + (size_t)T * dout * 2;
                    const bool have_edge = !imp && ib >= 0 && net->dz_edge[ib];  // dx_epilogue's
                    if (nl.compact && net->Tc) {
                        // compact rows: the source rows T-1-3 .. T-1 that are in the set, in
                        // source order (the others carry no gradient)
                        int rows[4], nr = 0;
                        for (int t = std::max(0, Tfull - 1 - L.time_stride); t < Tfull; ++t) {
                            const int c = compact_of(net, t);
                            if (c >= 0 && nr < 4) rows[nr++] = c;
                        }
                        if (!ck(kf_rows_sum_list(edge, dzs, dout, rows, nr, dout), "row set edge")) return -1;
                    } else if (!have_edge && !ck(kf_rows_sum_mask(edge, dzs, dout, T - 1 - s < 0 ? 0 : T - 1 - s, T, dout,
                                                                  imp ? nl.mask : nullptr),
                                                 "edge"))
                        return -1;
                    KfOperand B1 = op_wrows(w2, 2, bn, dout);
                    if (net->fp8 && i8 >= 0 && net->dz8_layer[i8] == li && T > 1) {
                        // MXFP8 (the one MFMA-bound backward product, K = 2 x dout): rows
                        // 0 .. T-2 from dz's e4m3 copy [dz(t) | dz(t-s)] against the e4m3
                        // weight rows; row T-1, whose second part is the clamped-edge sum,
                        // again in fp16 below (the MXFP8 operand has no edge rows)
                        const Mx &d8 = net->dz8[i8];
                        const int pw = pad128(dout);
                        KfOperand A1 = op_base(d8.q, d8.ld, T, 2 * pw, 1);
                        A1.nparts = 2;
                        A1.part_width = pw;
                        A1.dt[1] = -s;
                        A1.tpolicy = KF_ZERO;
                        A1.fmt = KF_FMT_MXFP8;
                        A1.scales = d8.s;
                        A1.lds = d8.ld / 32;
                        KfOperand B8 = op_mxw(nl.w8d, bn);
                        // rows 0 .. T-2, and row T-1 by the last row tile's workgroups
                        if (!ck(kf_gemm_fused_edge(T - 1, bn, 2 * pw, &A1, &B8, &E1,
                                                   (char *)dbott + (size_t)(T - 1) * bn * 2,
                                                   (const char *)dz + (size_t)(T - 1) * dout * 2, edge,
                                                   wptr(net, nl.pW2), dout),
                                "tdnnf affine dgrad mxfp8"))
                            return -1;
                    } else {
                        KfOperand A1 = masked(op_splice(dzs, T, dout, 0, -s, KF_ZERO, 1));
                        A1.edge_t[1] = T - 1;
                        A1.edge_row[1] = T;
                        if (!ck(kf_gemm_fused(T, bn, 2 * dout, &A1, &B1, &E1), "tdnnf affine dgrad"))
                            return -1;
                        if (zero_scratch)  // (no row mask for this bottleneck width)
                            bridge_gpu_memset((char *)dbott + (size_t)net->Tc0 * bn * 2, 0, (size_t)bn * 2);
                    }
                } else {
                    KfOperand A1 = masked(op_base(dzs, dout, T, dout, 1));
                    KfOperand B1 = op_base(w2, dout, bn, dout, 1);
                    if (!ck(kf_gemm_fused(T, bn, dout, &A1, &B1, &E1), "tdnnf affine dgrad")) return -1;
                }
                if (aff_on_main && !aff_wgrad()) return -1;
                // linear weight gradient: splice-(x)^T . dbott
                KfOperand A2 = s > 0 ? op_splice(x, T, din, -s, 0, KF_CLAMP, 0)
                                     : op_base(x, din, T, din, 0);
                KfOperand B2 = op_base(dbott, bn, T, bn, 0);
                if (!wgrad([&] {
                        return ck(kf_gemm_wgrad(klin, bn, T, &A2, &B2, gptr(net, nl.pW), bn, nullptr, 0),
                                  "tdnnf linear wgrad");
                    }))
                    return -1;
                if (want_dx) {
                    if (!dx_wait()) return -1;
                    // input gradient: transpose of the [-s, 0] clamped splice
                    if (s > 0) {
                        // spare row T of dbott holds sum_{t <= s} dbott[t]
                        // (row T of dbott: the affine input gradient's epilogue summed it, E1)
                        KfOperand A3 = op_splice(dbott, T, bn, s, 0, KF_ZERO, 1);
                        A3.edge_t[0] = 0;
                        A3.edge_row[0] = T;
                        KfOperand B3 = op_wrows(wptr(net, nl.pW), 2, din, bn);
                        if (!ck(kf_gemm_fused(T, din, 2 * bn, &A3, &B3, &E), "tdnnf linear dgrad"))
                            return -1;
                    } else {
                        KfOperand A3 = op_base(dbott, bn, T, bn, 1);
                        KfOperand B3 = op_base(wptr(net, nl.pW), bn, din, bn, 1);
                        if (!ck(kf_gemm_fused(T, din, bn, &A3, &B3, &E), "tdnnf linear dgrad")) return -1;
                    }
                }
                break;
            }
            case LayerType::ConvReluBN: {
                const int noff = (int)nl.dt.size();
                // compact-row conv (conv_compact): the input gradient of the frames from the
                // tail's reach up (ws - 1 ..., ws = first tail frame - 1) comes from the full-row
                // kernel on a window of the scattered output gradient dz (zero below it). It
                // runs first, on the weight-gradient stream (side = true) beside the residue GEMMs.
                auto conv_window = [&](bool side) -> bool {
                    const int nt = net->Tc - net->Tc0, ws = T - 1 - 3 * (nt - 1) - 1, tw = T - (ws - 1);
                    const long long fi = (long long)L.hin * L.fin, fo = (long long)L.hout * L.fout;
                    KfOperand A2 = op_col2im(nl, (const char *)dz + (ws - 1) * fo * 2, tw);
                    KfOperand B2 = op_wrows(wptr(net, nl.pW), noff, L.fin, L.fout);
                    KfEpilogue Ew = E;
                    Ew.ldo2 = L.fin;
                    Ew.out2 = (char *)E.out2 + (ws - 1) * fi * 2;
                    if (E.out) {
                        Ew.ldo = L.fin;
                        Ew.out = (char *)E.out + (ws - 1) * fi * 2;
                    }
                    if (E.mask_in) Ew.mask_in = E.mask_in + (ws - 1) * fi / 8;
                    if (side && !to_side()) return false;
                    const bool ok = ck(kf_gemm_fused(tw * L.hin, L.fin, noff * L.fout, &A2, &B2, &Ew),
                                       "conv dgrad (tail window)");
                    const bool rec = !side || kf_event_record(net->ev_aux, net->wg_stream) == 0;
                    if (side) to_main();
                    if (!rec) set_err("backward: conv window event");
                    return ok && rec;
                };
                if (want_dx && conv_compact(net, li) && net->Tc > net->Tc0 && two && E.out2 && !conv_window(true))
                    return -1;
                if (nl.kp) {  // small fin: the forward's im2col is still in nl.im2col
                    // wgrad over the padded K (the pad columns are zero), then the first
                    // ntaps*fin rows into the flat gradient
                    const int K = noff * L.fin;
                    KfOperand A = op_base(nl.im2col, nl.kp, T * L.hout, nl.kp, 0);
                    KfOperand B = op_base(dz, L.fout, T * L.hout, L.fout, 0);
                    if (!wgrad([&] {
                            return ck(kf_gemm_wgrad(nl.kp, L.fout, T * L.hout, &A, &B, nl.gwpad, L.fout,
                                                    gptr(net, nl.pb), 0),
                                      "conv small-fin wgrad") &&
                                   ck(ops_copy(gptr(net, nl.pW), nl.gwpad, 2 * K * L.fout), "conv small-fin wgrad copy");
                        }))
                        return -1;
                    if (want_dx) {
                        // the input gradient overwrites nl.im2col, which the weight gradient
                        // just read on side: main waits for side here
                        if (two && (kf_event_record(net->ev_side, net->wg_stream) != 0 ||
                                    kf_stream_wait(mainst, net->ev_side) != 0)) {
                            set_err("backward: weight-gradient stream join");
                            return -1;
                        }
                        joined();
                        if (E.out || E.mask_in || E.scale2 || !E.out2) {
                            set_err("conv " + L.name + ": small-fin input gradient only into combine-feature-maps");
                            return -1;
                        }
                        // dP = dz . Wpad^T into the im2col buffer, then the gather col2im
                        KfOperand A2 = op_base(dz, L.fout, T * L.hout, L.fout, 1);
                        KfOperand B2 = op_base(nl.wpad, L.fout, nl.kp, L.fout, 1);
                        KfEpilogue Ed = epi0();
                        Ed.out = nl.im2col;
                        Ed.ldo = nl.kp;
                        if (!ck(kf_gemm_fused(T * L.hout, nl.kp, L.fout, &A2, &B2, &Ed), "conv small-fin dgrad") ||
                            !ck(kf_col2im_small(nl.im2col, T, L.hin, L.hout, L.hsub, L.fin, noff, nl.dt.data(),
                                                nl.dh.data(), nl.kp, E.out2, din),
                                "col2im small"))
                            return -1;
                    }
                    break;
                }
                if (L.fin == 1) {
                    if (!wgrad([&] {
                            return ck(kf_conv_c1_wgrad(T, L.hin, L.hout, L.hsub, L.fout, noff, nl.dt.data(),
                                                       nl.dh.data(), x, dz, gptr(net, nl.pW), gptr(net, nl.pb)),
                                      "conv c1 wgrad");
                        }))
                        return -1;
                } else if (conv_compact(net, li)) {
                    // output gradient on the compact rows only (net->dzc): the reduction over
                    // output frames 3c (c < Tc0), then over the tail frames, added
                    const int nt = net->Tc - net->Tc0;
                    KfOperand A = op_im2col(nl, x, T, 0);
                    A.tmul = 3;
                    A.nrows = net->Tc0 * L.hout;
                    KfOperand B = op_base(net->dzc, L.fout, net->Tc0 * L.hout, L.fout, 0);
                    KfOperand At = A, Bt = B;
                    At.t0 = T - 1 - 3 * (nt - 1);
                    At.nrows = nt * L.hout;
                    Bt.base = (const char *)net->dzc + (size_t)net->Tc0 * L.hout * L.fout * 2;
                    Bt.nrows = Bt.T = nt * L.hout;
                    if (!wgrad([&] {
                            return ck(kf_gemm_wgrad(noff * L.fin, L.fout, net->Tc0 * L.hout, &A, &B, gptr(net, nl.pW),
                                                    L.fout, gptr(net, nl.pb), 0),
                                      "conv wgrad (compact rows)") &&
                                   (nt == 0 ||
                                    ck(kf_gemm_wgrad(noff * L.fin, L.fout, nt * L.hout, &At, &Bt, gptr(net, nl.pW),
                                                     L.fout, gptr(net, nl.pb), 1),
                                       "conv wgrad (compact tail rows)"));
                        }))
                        return -1;
                } else {
                    KfOperand A = op_im2col(nl, x, T, 0);
                    KfOperand B = op_base(dz, L.fout, T * L.hout, L.fout, 0);
                    if (!wgrad([&] {
                            return ck(kf_gemm_wgrad(noff * L.fin, L.fout, T * L.hout, &A, &B, gptr(net, nl.pW),
                                                    L.fout, gptr(net, nl.pb), 0),
                                      "conv wgrad");
                        }))
                        return -1;
                }
                if (want_dx) {
                    if (!dx_wait()) return -1;
                    if (L.fin == 1) {
                        set_err("conv " + L.name + ": input gradient of a 1-filter conv not supported");
                        return -1;
                    }
                    if (conv_compact(net, li)) {
                        if (!E.out2 || E.out8 || E.edge_out || E.resid || E.beta != 0.f) {
                            set_err("row subsampling: unsupported input gradient of " + L.name);
                            return -1;
                        }
                        // the output gradient is non-zero on the compact frames only (net->dzc):
                        // input frame f = 3c + e receives only the taps with dt = e, from compact
                        // frame c. One GEMM per residue e over those taps, its rows written to
                        // frames 3c + e in place (grouped epilogue rows); every nonzero term in
                        // the full-row kernel's order, so the result is bit-identical. The frames
                        // the tail reaches (from ws = first tail frame - 1) take the full-row
                        // kernel on a window of the scattered gradient dz (zero below it).
                        const int Tc0 = net->Tc0, nt = net->Tc - net->Tc0;
                        const int ws = nt > 0 ? T - 1 - 3 * (nt - 1) - 1 : T;
                        const long long fi = (long long)L.hin * L.fin, fo = (long long)L.hout * L.fout;
                        KfEpilogue Ep = E;
                        Ep.ldo2 = L.fin;
                        if (E.out) Ep.ldo = L.fin;
                        auto at_frame = [&](KfEpilogue &X, long long f) {
                            X.out2 = (char *)E.out2 + f * fi * 2;
                            if (E.out) X.out = (char *)E.out + f * fi * 2;
                            if (E.mask_in) X.mask_in = E.mask_in + f * fi / 8;
                            if (E.mask_out) X.mask_out = E.mask_out + f * fi / 8;
                        };
                        // (the tail window, frames ws - 1 .., went to the weight-gradient stream at
                        // the start of this step, conv_window; the residue GEMMs take frames
                        // below it, and main joins the window after them)
                        const bool wside = nt > 0 && two;
                        if (nt > 0 && !two && !conv_window(false)) return -1;
                        const int flim = nt > 0 ? ws - 2 : T - 1;  // the last frame of the residues
                        for (int e = -1; e <= 1; ++e) {
                            const int c_hi = std::min(Tc0, (flim - e) / 3 + 1), c_lo = e < 0 ? 1 : 0;
                            if (c_hi <= c_lo) continue;
                            KfOperand A2 = op_col2im(nl, (const char *)net->dzc + c_lo * fo * 2, c_hi - c_lo);
                            KfOperand B2 = op_wrows(wptr(net, nl.pW), noff, L.fin, L.fout);
                            int np = 0;
                            for (int o = 0; o < noff; ++o) {
                                if (nl.dt[o] != e) continue;
                                A2.dt[np] = 0;
                                A2.dh[np] = -nl.dh[o];
                                B2.dt[np] = o * L.fin;
                                ++np;
                            }
                            A2.nparts = B2.nparts = np;
                            A2.ncols = B2.ncols = np * L.fout;
                            KfEpilogue Er = Ep;
                            at_frame(Er, 3LL * c_lo + e);
                            Er.row_group = L.hin;
                            Er.row_stride = 3 * L.hin;
                            if (!ck(kf_gemm_fused((c_hi - c_lo) * L.hin, L.fin, np * L.fout, &A2, &B2, &Er),
                                    "conv dgrad (compact rows)"))
                                return -1;
                        }
                        if (wside && kf_stream_wait(mainst, net->ev_aux) != 0) {
                            set_err("backward: conv window join");
                            return -1;
                        }
                    } else if (L.hsub > 1 && L.hin % L.hsub == 0 && !E.out && hsub_merge(net, nl)) {
                        // strided conv, every residue in one GEMM of N = hsub * fin columns: the
                        // output row (t, j) holds input rows h' = hsub*j + pi, pi < hsub, which is
                        // the [(t,h) x fin] gradient itself. Part p = (dt, dh') of the merged list;
                        // the weight block of (p, pi) is the tap o with dh_o = pi - hsub*dh', or
                        // zeros. Each residue's taps keep their order in K (hsub_merge), and the
                        // zero blocks add exact zeros, so every column sums the per-residue
                        // GEMM's terms in its order.
                        const int np = nl.wm_np;
                        if (!ck(kf_copy_blocks(nl.wm, wptr(net, nl.pW), (long long)L.fin * L.fout * 2, nl.wm_map.data(),
                                               np * L.hsub),
                                "conv dgrad (strided, merged weights)"))
                            return -1;
                        KfOperand A2 = op_col2im(nl, dz, T);
                        KfOperand B2 = op_wrows(nl.wm, np, L.hsub * L.fin, L.fout);
                        for (int p = 0; p < np; ++p) {
                            A2.dt[p] = -nl.wm_dt[p];
                            A2.dh[p] = nl.wm_dh[p];
                        }
                        A2.nparts = B2.nparts = np;
                        A2.ncols = B2.ncols = np * L.fout;
                        A2.hout = L.hin / L.hsub;
                        A2.hmul = 1;
                        A2.hdiv = 1;
                        A2.nrows = T * A2.hout;
                        KfEpilogue Ep = E;
                        Ep.ldo2 = (long long)L.hsub * L.fin;
                        if (!ck(kf_gemm_fused(T * A2.hout, L.hsub * L.fin, np * L.fout, &A2, &B2, &Ep),
                                "conv dgrad (strided, merged)"))
                            return -1;
                    } else if (L.hsub > 1 && L.hin % L.hsub == 0 && !E.out) {
                        // strided conv: input row h' = hsub*j + pi only receives the taps
                        // with (pi - dh) % hsub == 0, so one GEMM per residue pi skips the
                        // (hsub-1)/hsub of the K range the plain col2im reads as zeros
                        const bool twt = dgrad_wt_on();
                        std::vector<int> taps;  // every residue's taps, residue by residue
                        for (int pi = 0; pi < L.hsub; ++pi)
                            for (int o = 0; o < noff; ++o)
                                if (!((((pi - nl.dh[o]) % L.hsub) + L.hsub) % L.hsub)) taps.push_back(o);
                        char *wt = nullptr;
                        if (twt && !(wt = (char *)dgrad_wt(net, nl, taps))) {
                            set_err("conv dgrad (strided): transposed weights of " + L.name);
                            return -1;
                        }
                        int tap0 = 0;  // the residue's first block in wt
                        for (int pi = 0; pi < L.hsub; ++pi) {
                            KfOperand A2 = op_col2im(nl, dz, T);
                            KfOperand B2 = op_wrows(wptr(net, nl.pW), noff, L.fin, L.fout);
                            int np = 0;
                            for (int o = 0; o < noff; ++o) {
                                const int r = pi - nl.dh[o];
                                if (((r % L.hsub) + L.hsub) % L.hsub) continue;
                                A2.dt[np] = -nl.dt[o];
                                A2.dh[np] = r / L.hsub;  // exact: r is a multiple of hsub
                                B2.dt[np] = o * L.fin;
                                ++np;
                            }
                            if (!np) continue;
                            A2.nparts = B2.nparts = np;
                            A2.ncols = B2.ncols = np * L.fout;
                            if (twt) B2 = op_base(wt + (size_t)tap0 * L.fin * L.fout * 2, L.fin, np * L.fout, L.fin, 0);
                            tap0 += np;
                            A2.hout = L.hin / L.hsub;
                            A2.hmul = 1;
                            A2.hdiv = 1;
                            A2.nrows = T * A2.hout;
                            KfEpilogue Ep = E;  // rows hsub*m + pi of the [(t,h) x fin] gradient
                            Ep.out2 = (char *)E.out2 + (size_t)pi * L.fin * 2;
                            Ep.ldo2 = (long long)L.hsub * L.fin;
                            if (E.mask_in) Ep.mask_in = E.mask_in + (size_t)pi * L.fin / 8;
                            if (!ck(kf_gemm_fused(T * A2.hout, L.fin, np * L.fout, &A2, &B2, &Ep),
                                    "conv dgrad (strided)"))
                                return -1;
                        }
                    } else {
                        KfOperand A2 = op_col2im(nl, dz, T);
                        KfOperand B2 = op_wrows(wptr(net, nl.pW), noff, L.fin, L.fout);
                        if (dgrad_wt_on()) {
                            std::vector<int> taps(noff);
                            for (int o = 0; o < noff; ++o) taps[o] = o;
                            void *wt = dgrad_wt(net, nl, taps);
                            if (!wt) {
                                set_err("conv dgrad: transposed weights of " + L.name);
                                return -1;
                            }
                            B2 = op_base(wt, L.fin, noff * L.fout, L.fin, 0);
                        }
                        E.ldo2 = L.fin;  // dz of the input conv layer viewed as [(t,h) x fin]
                        if (E.out) E.ldo = L.fin;
                        if (!ck(kf_gemm_fused(T * L.hin, L.fin, noff * L.fout, &A2, &B2, &E), "conv dgrad"))
                            return -1;
                    }
                }
                break;
            }
            case LayerType::CombineFeatureMaps:
                if (nl.input2 >= 0 && net->layers[nl.input2].needs_dx + is_trainable(net->layers[nl.input2].L.type)) {
                    // the ivector branch: sum the broadcast columns per sequence, then back
                    // through its batchnorm-component(s) and linear-component (B rows)
                    const bool bseq = net->layers[nl.input2].per_seq;
                    if (!bseq) {
                        set_err("combine " + L.name + ": gradient into a frame-level second input not supported");
                        return -1;
                    }
                    const int wb = L.height * L.nf2, rowsB = net->B;
                    if (!ck(kf_combine_feature_maps_backward(dz, dout, net->seq_off, rowsB, nl.gdb, wb, L.height,
                                                             L.nf1, L.nf2),
                            "combine backward"))
                        return -1;
                    int cur = nl.input2;
                    while (cur >= 0) {
                        NetLayer &q = net->layers[cur];
                        const int qd = q.L.out_dim;
                        if (q.L.type == LayerType::Batchnorm) {
                            if (!ck(kf_scale_cols(nl.gdb, qd, q.bn_scale, nl.gdb, qd, rowsB, qd), "ivector bn backward"))
                                return -1;
                        } else if (q.L.type == LayerType::Linear) {
                            if (!wgrad([&] {
                                    return ck(kf_rows_wgrad(act_of(net, q.input), q.L.in_dim, nl.gdb, qd,
                                                            gptr(net, q.pW), qd, rowsB, q.L.in_dim, qd),
                                              "ivector linear wgrad");
                                }))
                                return -1;
                            if (q.input >= 0) {
                                set_err("ivector branch: a linear-component below another one is not supported");
                                return -1;
                            }
                        } else {
                            set_err("ivector branch: unsupported layer " + q.L.name);
                            return -1;
                        }
                        cur = q.input;
                    }
                }
                if (nl.needs_dx && nl.input >= 0 && net->layers[nl.input].needs_dx +
                                                        is_trainable(net->layers[nl.input].L.type)) {
                    set_err("backward through " + L.name + " into a trainable frame-level input is not supported");
                    return -1;
                }
                want_dx = false;
                break;
            case LayerType::Batchnorm:
                if (want_dx) {  // dz already is the gradient at the BN input (dx_epilogue)
                    if (net->dp && !wgrad([&] { return dp_issue(net, dp_next, done); })) return -1;
                    continue;   // same dz / gcur buffers for the layer below: no flip
                }
                break;
            case LayerType::IDCT:
            case LayerType::SpecAugment:
                if (want_dx) {
                    set_err("backward through " + L.name + " into trainable layers is not supported");
                    return -1;
                }
                break;
            default:
                set_err("backward: unsupported layer " + L.name);
                return -1;
        }
        if (want_dx && to_full) {
            const int w = net->layers[nl.input].L.out_dim;
            if (net->conv_c) {
                // the conv below reads the compact rows (net->dzc); only its tail window
                // (full rows from ws - 1, conv_dx_window) takes the scattered form
                const int nt = net->Tc - net->Tc0;
                const int r0 = Tfull - 1 - 3 * (nt - 1) - 2;
                if (nt > 0 && !ck(kf_scatter_rows_from((char *)dz_next + (size_t)r0 * w * 2, net->dzc,
                                                       (long long)w * 2, Tfull, net->Tc0, net->Tc, r0),
                                  "row set scatter (tail window)"))
                    return -1;
            } else if (!ck(kf_scatter_rows(dz_next, net->dzc, (long long)w * 2, Tfull, net->Tc0, net->Tc),
                           "row set scatter")) {
                return -1;
            }
        }
        // gradient buckets complete at this step go to the communication stream (their
        // gates on side, behind the step's weight gradients)
        if (two) kf_set_stream(net->wg_stream);
        if (net->dp && !dp_issue(net, dp_next, done)) return -1;
        if (two) {
            if (kf_event_record(net->ev_step[stepi % 3], net->wg_stream) != 0) {
                set_err("backward: weight-gradient stream event");
                return -1;
            }
        }
        to_main();
        if (!want_dx) break;  // nothing trainable below
        dz = dz_next;
        gcur = g_next;
        net->dz_last = dz_next;
        ++stepi;
        flip = stepi % 3;
    }
    // the rest of the buckets, then main waits for side (SGD reads every gradient) and for
    // every bucket
    if (two) kf_set_stream(net->wg_stream);
    if (net->dp && !dp_issue(net, dp_next, INT_MAX)) return -1;
    to_main();
    if (two && (kf_event_record(net->ev_side, net->wg_stream) != 0 || kf_stream_wait(mainst, net->ev_side) != 0)) {
        set_err("backward: weight-gradient stream join");
        return -1;
    }
    if (hp) {  // the caller's stream continues after the chain (which joined side)
        if (kf_event_record(net->ev_go, mainst) != 0 || kf_stream_wait(caller, net->ev_go) != 0) {
            set_err("backward: chain stream join");
            return -1;
        }
        mainst = caller;
        kf_set_stream(caller);
    }
    if (net->dp && kf_dp_join(net->dp) != 0) {
        set_err(std::string("dp join: ") + (kf_dp_last_error() ? kf_dp_last_error() : ""));
        return -1;
    }
    return 0;
}

extern "C" int nnet_set_implicit_dz(KfNet *net, int on) {
    if (!net) return -1;
    net->implicit_dz = on != 0;
    return 0;
}

extern "C" int nnet_set_row_subsampling(KfNet *net, int stride) {
    if (!on_device(net, "set_row_subsampling")) return -1;
    if (stride == 0 || stride == 1) {
        net->rsub = 0;
        return 0;
    }
    if (stride != 3) {
        set_err("set_row_subsampling: stride " + std::to_string(stride) + " (only 3: chain frame subsampling)");
        return -1;
    }
    // the top of the output chain whose rows are row-local or 3-strided: TDNN-F with time
    // stride 0 or 3, linear, prefinal, output; consecutive layers. Every layer after the
    // first of them is such a layer too (e.g. Kaldi's xent branch, prefinal-xent and
    // output-xent on prefinal-l), and nothing below reads them.
    const int n = (int)net->layers.size();
    auto row_local = [&](const NetLayer &nl) {
        const Layer &L = nl.L;
        return (L.type == LayerType::TDNNF && (L.time_stride == 0 || L.time_stride == 3)) ||
               (L.type == LayerType::Linear && !nl.per_seq) || L.type == LayerType::Prefinal ||
               L.type == LayerType::Output;
    };
    int first = -1, n3 = 0;
    for (int li = net->chain_out; li >= 0; li = net->layers[li].input) {
        const NetLayer &nl = net->layers[li];
        if (!row_local(nl) || nl.input != li - 1) break;
        first = li;
        if (nl.L.type == LayerType::TDNNF && nl.L.time_stride == 3) ++n3;
    }
    if (first < 0 || net->layers[first].input < 0 || net->layers[net->layers[first].input].L.type != LayerType::ConvReluBN) {
        set_err("set_row_subsampling: needs row-local / 3-strided layers above a conv-relu-batchnorm layer");
        return -1;
    }
    for (int li = first; li < n; ++li)
        if (!row_local(net->layers[li]) || (net->layers[li].input >= 0 && net->layers[li].input < first - 1) ||
            net->layers[li].input2 > -100) {
            set_err("set_row_subsampling: layer " + net->layers[li].L.name + " above the row set is not row-local");
            return -1;
        }
    for (int li = 0; li < first; ++li)
        if (net->layers[li].input >= first || net->layers[li].input2 >= first) {
            set_err("set_row_subsampling: layer " + net->layers[li].L.name + " reads a layer of the row set");
            return -1;
        }
    // tail depth: one row per 3-strided layer and a margin (the scratch row's reach)
    const int nt = n3 + 4;
    const int maxTc = (net->max_T - 1) / 3 + 1 + nt;
    const int din = net->layers[first].L.in_dim;
    if (!net->xc || net->maxTc < maxTc || net->first_c != first) {
        net->xc = net->dalloc((size_t)maxTc * din * 2);
        net->dzc = net->dalloc((size_t)(maxTc + 2) * din * 2);
        net->mc = (uint8_t *)net->dalloc(align_up((size_t)maxTc * din / 8 + 16, 256));
        int maxbn = 0;
        for (int li = first; li < n; ++li)
            if (net->layers[li].L.type == LayerType::TDNNF) maxbn = std::max(maxbn, net->layers[li].L.bottleneck);
        net->rowmask = maxbn ? (uint8_t *)net->dalloc(align_up((size_t)maxTc * maxbn / 8 + 16, 256)) : nullptr;
        net->rm_bn = 0;
        net->rm_tc0 = net->rm_tc = -1;
        if (!net->xc || !net->dzc || !net->mc) {
            set_err("set_row_subsampling: alloc compact buffers");
            return -1;
        }
    }
    for (int li = 0; li < n; ++li) net->layers[li].compact = li >= first;
    net->first_c = first;
    {
        const NetLayer &cl = net->layers[net->layers[first].input];
        const char *ev = getenv("KF_RSUB_CONV");
        // time offsets exactly {-1, 0, 1} and no height subsampling: the input gradient's
        // per-residue GEMMs (backward) cover every input frame
        bool dt3 = !cl.dt.empty();
        for (int e = -1; e <= 1 && dt3; ++e) dt3 = std::find(cl.dt.begin(), cl.dt.end(), e) != cl.dt.end();
        for (int d : cl.dt) dt3 = dt3 && d >= -1 && d <= 1;
        net->conv_c = cl.L.fin > 1 && !cl.kp && cl.L.hsub == 1 && dt3 && !(ev && ev[0] == '0');
        for (int li = 0; li < n; ++li)  // first_c must be the conv output's only reader
            if (li != first && (net->layers[li].input == net->layers[first].input ||
                                net->layers[li].input2 == net->layers[first].input))
                net->conv_c = 0;
    }
    net->rs_nt = nt;
    net->maxTc = maxTc;
    net->rsub = 3;
    return 0;
}

extern "C" int nnet_row_set(const KfNet *net, int *tc, int *tc0) {
    if (!net) return -1;
    if (tc) *tc = net->Tc;
    if (tc0) *tc0 = net->Tc0;
    return 0;
}

extern "C" int nnet_debug_backward(KfNet *net, int main_aff, long long stall_cycles) {
    if (!net || main_aff < -1 || main_aff > 2 || stall_cycles < 0) return -1;
    net->main_aff = main_aff;
    net->stall_side = stall_cycles;
    return 0;
}

extern "C" int nnet_set_wgrad_stream(KfNet *net, int on) {
    if (!net) return -1;
    if (!on && net->wg_stream) bridge_gpu_sync();
    net->wg_side = on != 0 && net->wg_stream != nullptr;
    return 0;
}

extern "C" float *nnet_grad_buffer(KfNet *net) { return net->grad; }
extern "C" float *nnet_master_buffer(KfNet *net) { return net->master; }
extern "C" void *nnet_weight_buffer(KfNet *net) {
    net->wt_dirty = true;  // the caller may write the weights through it
    return net->w16;
}

extern "C" int nnet_weights_changed(KfNet *net) {
    if (!on_device(net, "weights_changed")) return -1;
    net->wt_dirty = true;  // the transposed copies are refreshed at the next forward
    return net->fp8 && !quantise_weights(net, false) ? -1 : 0;
}

extern "C" int nnet_sgd(KfNet *net, float lr, float momentum) {
    kf_take_pending(__func__);
    if (!on_device(net, "sgd")) return -1;
    if (!ck(kf_sgd_flat(net->master, net->w16, net->grad, net->vel, lr, momentum, net->nparams), "sgd"))
        return -1;
    net->wt_dirty = true;
    // the MXFP8 weight copies follow every parameter change
    return net->fp8 && !quantise_weights(net, false) ? -1 : 0;
}

// Parse + resolve only (no device work): one line per layer
// "name type in_dim out_dim" followed by "params N". Returns bytes needed, -1 on error.
extern "C" int nnet_parse_summary(const char *xconfig_text, char *out, int outlen) {
    std::vector<kf::LayerConfig> cfgs;
    std::vector<Layer> layers;
    std::string err;
    if (!kf::ParseXConfig(xconfig_text ? xconfig_text : "", cfgs, err) ||
        !kf::ResolveLayers(cfgs, layers, err)) {
        set_err("parse xconfig: " + err);
        return -1;
    }
    std::string s;
    long long nparams = 0;
    for (const Layer &L : layers) {
        s += L.name + " " + std::to_string((int)L.type) + " " + std::to_string(L.in_dim) + " " +
             std::to_string(L.out_dim) + "\n";
        switch (L.type) {
            case LayerType::ConvReluBN:
                nparams += (long long)L.time_offsets.size() * L.height_offsets.size() * L.fin * L.fout + L.fout;
                break;
            case LayerType::TDNNF: {
                int k = L.time_stride > 0 ? 2 : 1;
                nparams += (long long)k * L.in_dim * L.bottleneck + (long long)k * L.bottleneck * L.out_dim + L.out_dim;
                break;
            }
            case LayerType::Linear: nparams += (long long)L.in_dim * L.out_dim; break;
            case LayerType::Prefinal:
                nparams += (long long)L.in_dim * L.big_dim + L.big_dim + (long long)L.big_dim * L.small_dim;
                break;
            case LayerType::Output: nparams += (long long)L.in_dim * L.out_dim + L.out_dim; break;
            default: break;
        }
    }
    s += "params " + std::to_string(nparams) + "\n";
    if (out && outlen > 0) snprintf(out, outlen, "%s", s.c_str());
    return (int)s.size() + 1;
}

// Use caller-owned device memory (>= num_params fp32) as the gradient buffer,
// e.g. a torch tensor handed to the data-parallel all-reduce.
extern "C" int nnet_bind_grad_buffer(KfNet *net, float *dev) {
    if (!on_device(net, "bind_grad_buffer")) return -1;
    if (!dev) {
        set_err("bind_grad_buffer: null");
        return -1;
    }
    net->grad = dev;
    return 0;
}

// ---------------------------------------------------------------------------
// data parallel (kf_dp.h): the backward's parameter groups in the
// order backward_impl visits them, cut into all-reduce buckets by kf_dp_plan
// ---------------------------------------------------------------------------
namespace {
// [lo, hi) of the flat buffer written by backward step i (lo = hi: none)
void backward_groups(const KfNet *net, std::vector<long long> &lo, std::vector<long long> &hi) {
    lo.clear();
    hi.clear();
    auto add = [&](const NetLayer &q, long long &a, long long &b) {
        for (int pi : {q.pW, q.pb, q.pW2, q.pb2}) {
            if (pi < 0) continue;
            const ParamRef &p = net->params[pi];
            const long long e = p.off + (long long)align_up((size_t)p.rows * p.cols, 64);
            if (a == b) {
                a = p.off;
                b = e;
            } else {
                a = std::min(a, p.off);
                b = std::max(b, e);
            }
        }
    };
    for (int li = net->chain_out; li >= 0; li = net->layers[li].input) {
        const NetLayer &nl = net->layers[li];
        long long a = 0, b = 0;
        add(nl, a, b);
        if (nl.L.type == LayerType::CombineFeatureMaps)  // the ivector branch is written at this step
            for (int cur = nl.input2; cur >= 0; cur = net->layers[cur].input) add(net->layers[cur], a, b);
        lo.push_back(a);
        hi.push_back(b);
    }
}
}  // namespace

extern "C" int nnet_dp_plan(const KfNet *net, long long bucket_bytes, int max_buckets, int *after_step,
                            long long *begin, long long *end) {
    if (!net || bucket_bytes < 0) {
        set_err("dp_plan: bad arguments");
        return -1;
    }
    std::vector<long long> lo, hi;
    backward_groups(net, lo, hi);
    const int nb = kf_dp_plan((int)lo.size(), lo.data(), hi.data(), net->nparams, bucket_bytes / 4, max_buckets,
                              after_step, begin, end);
    if (nb < 0) set_err(std::string("dp_plan: ") + (kf_dp_last_error() ? kf_dp_last_error() : ""));
    return nb;
}

extern "C" int nnet_bind_dp(KfNet *net, KfDp *dp, long long bucket_bytes) {
    if (!on_device(net, "bind_dp")) return -1;
    net->dp = nullptr;
    net->dp_after.clear();
    net->dp_begin.clear();
    net->dp_end.clear();
    if (!dp) return 0;
    std::vector<int> after(256);
    std::vector<long long> b(256), e(256);
    const int nb = nnet_dp_plan(net, bucket_bytes, 256, after.data(), b.data(), e.data());
    if (nb < 0) return -1;
    net->dp_after.assign(after.begin(), after.begin() + nb);
    net->dp_begin.assign(b.begin(), b.begin() + nb);
    net->dp_end.assign(e.begin(), e.begin() + nb);
    net->dp = dp;
    return 0;
}

extern "C" int nnet_dp_debug_early(KfNet *net, int on) {
    if (!net) return -1;
    net->dp_early = on != 0;
    return 0;
}

// issue every bucket planned to follow backward step `step` (INT_MAX: all left)
static bool dp_issue(KfNet *net, size_t &next, int step) {
    for (; next < net->dp_after.size() && net->dp_after[next] <= step; ++next)
        if (kf_dp_allreduce_mean_async(net->dp, net->grad + net->dp_begin[next],
                                       (size_t)(net->dp_end[next] - net->dp_begin[next])) != 0) {
            const char *e = kf_dp_last_error();
            set_err(std::string("dp all-reduce: ") + (e ? e : ""));
            return false;
        }
    return true;
}
