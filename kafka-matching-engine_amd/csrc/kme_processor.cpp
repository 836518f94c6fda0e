// kme_processor.cpp -- the Processor<String, Order> mirror over the epoch engine (kme.h).
#include "kme_processor.hpp"

#include <algorithm>
#include <cstring>

#include "kme_processor.h"

namespace kme {

MatchingEngine::MatchingEngine(const kme_config& cfg, uint32_t epoch_records)
    : cfg_(cfg), epoch_records_(epoch_records ? epoch_records : 1) {
    if (epoch_records_ > cfg_.max_epoch) epoch_records_ = cfg_.max_epoch;
}

MatchingEngine::~MatchingEngine() {
    if (engine_) kme_destroy(engine_);
}

// init (KP:86-93): the stores are created on the device and bound to this instance.
void MatchingEngine::init(ProcessorContext* context) {
    context_ = context;
    const kme_status rc = kme_create(&cfg_, &engine_);
    if (rc != KME_OK) {
        kme_epoch_status st{};
        st.status = rc;
        st.error_index = -1;
        throw EngineError(rc, st, std::string("kme_create: ") + kme_strerror(rc));
    }
    action_.reserve(epoch_records_);
}

// process (KP:96): buffer; the epoch is matched and forwarded once full.
void MatchingEngine::process(const std::string& /*key ignored, KP:96*/, const Order& o) {
    if (dead_) throw EngineError(KME_E_FAILED, last_, "processor is dead");
    if (o.next || o.prev) {
        dead_ = true;
        kme_epoch_status st{};
        st.status = KME_E_DOMAIN;
        st.error_index = stream_base_ + (int64_t)action_.size();
        throw EngineError(KME_E_DOMAIN, st, "input Order with next/prev links is outside the parity domain");
    }
    action_.push_back(o.action); oid_.push_back(o.oid); aid_.push_back(o.aid); sid_.push_back(o.sid);
    price_.push_back(o.price); size_.push_back(o.size);
    if (action_.size() >= epoch_records_) flush();
}

void MatchingEngine::punctuate() {
    if (dead_) throw EngineError(KME_E_FAILED, last_, "processor is dead");
    flush();
}

// close (KP:129): drain what is buffered, then release the device stores.
void MatchingEngine::close() {
    if (!dead_ && !action_.empty()) flush();
    if (engine_) { kme_destroy(engine_); engine_ = nullptr; }
}

void MatchingEngine::flush() {
    const uint32_t n = (uint32_t)action_.size();
    if (n == 0) return;
    out_action_.resize(n); out_size_.resize(n); out_prev_.resize(n); out_flags_.resize(n);
    trade_off_.resize((size_t)n + 1);
    if (trades_.size() < cfg_.max_trades) trades_.resize(cfg_.max_trades);
    kme_orders in{action_.data(), oid_.data(), aid_.data(), sid_.data(), price_.data(), size_.data()};
    kme_epoch_result res{out_action_.data(), out_size_.data(), out_prev_.data(), out_flags_.data(),
                         trade_off_.data(), trades_.data(), (uint32_t)trades_.size()};
    const kme_status rc = kme_submit_epoch(engine_, &in, n, &res, &last_);
    if (rc != KME_OK) {
        // The reference forwards and commits every record before the one that throws (KP:97,
        // 124-125) and then its stream thread dies: forward the records that took effect, commit
        // them, then fail.  (Records the reference had forwarded for the faulting record itself --
        // its IN echo, fills before the throw -- are not: whether its producer flushed them when
        // the thread died is outside what the reference pins.)
        forward_range(std::min<uint32_t>(last_.n_effective, n));
        if (last_.n_effective > 0) context_->commit();
        dead_ = true;
        if (last_.error_index >= 0) last_.error_index += stream_base_;
        throw EngineError(rc, last_, std::string("epoch failed: ") + kme_strerror(rc) + " (" +
                                         kme_domain_str(last_.detail) + ")");
    }
    forward_range(n);
    context_->commit();
    stream_base_ += n;
    action_.clear(); oid_.clear(); aid_.clear(); sid_.clear(); price_.clear(); size_.clear();
}

void MatchingEngine::forward_range(uint32_t n) {
    // Forward in the reference's order: IN, (maker fill, taker fill) per trade, OUT (KP:97-124).
    for (uint32_t i = 0; i < n; ++i) {
        Order in_o;
        in_o.action = action_[i]; in_o.oid = oid_[i]; in_o.aid = aid_[i]; in_o.sid = sid_[i];
        in_o.price = price_[i]; in_o.size = size_[i];
        context_->forward("IN", in_o);
        const bool taker_buy = action_[i] == KME_BUY;
        for (uint32_t t = trade_off_[i]; t < trade_off_[i + 1]; ++t) {
            const kme_trade& tr = trades_[t];
            Order mk;   // executeTrade maker fill (KP:266-267)
            mk.action = taker_buy ? KME_SOLD : KME_BOUGHT;
            mk.oid = tr.maker_oid; mk.aid = tr.maker_aid; mk.sid = tr.maker_sid; mk.price = 0; mk.size = tr.size;
            context_->forward("OUT", mk);
            Order tk;   // executeTrade taker fill (KP:268-269)
            tk.action = taker_buy ? KME_BOUGHT : KME_SOLD;
            tk.oid = oid_[i]; tk.aid = aid_[i]; tk.sid = sid_[i];
            tk.price = (int32_t)((uint32_t)price_[i] - (uint32_t)tr.maker_price);
            tk.size = tr.size;
            context_->forward("OUT", tk);
        }
        Order out_o = in_o;   // the mutated input (KP:123-124)
        out_o.action = out_action_[i];
        out_o.size = out_size_[i];
        if (out_flags_[i] & KME_OUT_HAS_PREV) out_o.prev = out_prev_[i];
        context_->forward("OUT", out_o);
    }
}

}  // namespace kme

// ------------------------------------------------------------------ C ABI (kme_processor.h)
namespace {

char* put_i64(char* p, int64_t v) {
    char tmp[24];
    int n = 0;
    uint64_t u = v < 0 ? (0ull - (uint64_t)v) : (uint64_t)v;
    do { tmp[n++] = (char)('0' + (u % 10)); u /= 10; } while (u);
    if (v < 0) *p++ = '-';
    while (n) *p++ = tmp[--n];
    return p;
}
char* put_opt(char* p, const std::optional<int64_t>& v) {
    if (v) return put_i64(p, *v);
    std::memcpy(p, "null", 4);
    return p + 4;
}
char* put_s(char* p, const char* s) {
    const size_t n = std::strlen(s);
    std::memcpy(p, s, n);
    return p + n;
}

// The MatchOut sink: JsonSerializer<Order> (KP:488-494) then the user's callback.
class JsonSinkContext : public kme::ProcessorContext {
public:
    JsonSinkContext(kme_forward_fn f, kme_commit_fn c, void* u) : f_(f), c_(c), u_(u) {}
    void forward(const std::string& key, const kme::Order& o) override {
        char buf[320];
        char* p = buf;
        p = put_s(p, "{\"action\":"); p = put_i64(p, o.action);
        p = put_s(p, ",\"oid\":"); p = put_i64(p, o.oid);
        p = put_s(p, ",\"aid\":"); p = put_i64(p, o.aid);
        p = put_s(p, ",\"sid\":"); p = put_i64(p, o.sid);
        p = put_s(p, ",\"price\":"); p = put_i64(p, o.price);
        p = put_s(p, ",\"size\":"); p = put_i64(p, o.size);
        p = put_s(p, ",\"next\":"); p = put_opt(p, o.next);
        p = put_s(p, ",\"prev\":"); p = put_opt(p, o.prev);
        *p++ = '}';
        *p = 0;
        if (f_) f_(u_, key.c_str(), buf, (size_t)(p - buf));
    }
    void commit() override { if (c_) c_(u_); }

private:
    kme_forward_fn f_;
    kme_commit_fn c_;
    void* u_;
};

}  // namespace

struct kme_processor {
    JsonSinkContext ctx;
    kme::MatchingEngine engine;
    kme_epoch_status last{};
    kme_processor(const kme_config& cfg, uint32_t epoch, kme_forward_fn f, kme_commit_fn c, void* u)
        : ctx(f, c, u), engine(cfg, epoch) {}
};

extern "C" {

kme_status kme_processor_create(const kme_config* cfg, uint32_t epoch_records, kme_forward_fn forward,
                                kme_commit_fn commit, void* user, kme_processor** out) {
    if (!cfg || !out) return KME_E_INVALID;
    kme_processor* p = new kme_processor(*cfg, epoch_records, forward, commit, user);
    try {
        p->engine.init(&p->ctx);
    } catch (const kme::EngineError& e) {
        delete p;
        return (kme_status)e.status();
    }
    *out = p;
    return KME_OK;
}

static kme_status guarded(kme_processor* p, const kme::Order& o) {
    try {
        p->engine.process("", o);
    } catch (const kme::EngineError& e) {
        p->last = e.epoch_status();
        return (kme_status)e.status();
    }
    return KME_OK;
}

kme_status kme_processor_process_json(kme_processor* p, const char* json, size_t len) {
    if (!p || !json) return KME_E_INVALID;
    kme::Order o;
    const kme_status rc = kme_order_from_json(json, len, &o.action, &o.oid, &o.aid, &o.sid, &o.price, &o.size);
    if (rc != KME_OK) return rc;
    return guarded(p, o);
}

kme_status kme_processor_process(kme_processor* p, int32_t action, int64_t oid, int64_t aid, int64_t sid,
                                 int32_t price, int32_t size) {
    if (!p) return KME_E_INVALID;
    kme::Order o;
    o.action = action; o.oid = oid; o.aid = aid; o.sid = sid; o.price = price; o.size = size;
    return guarded(p, o);
}

kme_status kme_processor_punctuate(kme_processor* p) {
    if (!p) return KME_E_INVALID;
    try {
        p->engine.punctuate();
    } catch (const kme::EngineError& e) {
        p->last = e.epoch_status();
        return (kme_status)e.status();
    }
    p->last = p->engine.last_status();
    return KME_OK;
}

kme_status kme_processor_close(kme_processor* p) {
    if (!p) return KME_E_INVALID;
    kme_status rc = KME_OK;
    try {
        p->engine.close();
    } catch (const kme::EngineError& e) {
        rc = (kme_status)e.status();
    }
    delete p;
    return rc;
}

kme_status kme_processor_last_status(kme_processor* p, kme_epoch_status* st) {
    if (!p || !st) return KME_E_INVALID;
    *st = p->last;
    return KME_OK;
}

}  // extern "C"
