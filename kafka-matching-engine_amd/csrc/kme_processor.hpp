// kme_processor.hpp -- C++ mirror of the reference's processor API for the matching path.
//
// Same names and contract as KProcessor.MatchingEngine (/root/reference/src/main/java/
// KProcessor.java:63-129) and the Kafka Streams 2.3 Processor/ProcessorContext it implements:
//   init(ProcessorContext*)          KP:86-93
//   process(key, Order)              KP:96-126  (buffered into epochs of the device engine)
//   punctuate()                      the epoch flush a Punctuator would trigger
//   close()                          KP:129
// Errors mirror the reference's failure mode: where the reference would throw (and kill the
// stream thread), process()/punctuate() throw kme::EngineError and the processor stays dead.
#pragma once
#include <cstdint>
#include <optional>
#include <stdexcept>
#include <string>
#include <vector>

#include "kme.h"

namespace kme {

struct Order {                       // Order, KP:449-458
    int32_t action = 0;
    int64_t oid = 0, aid = 0, sid = 0;
    int32_t price = 0, size = 0;
    std::optional<int64_t> next, prev;
};

class ProcessorContext {             // the subset of ProcessorContext the path uses
public:
    virtual ~ProcessorContext() = default;
    virtual void forward(const std::string& key, const Order& value) = 0;   // KP:97, 124, 272-273
    virtual void commit() = 0;                                              // KP:125
};

class EngineError : public std::runtime_error {
public:
    EngineError(int status, const kme_epoch_status& st, const std::string& what)
        : std::runtime_error(what), status_(status), st_(st) {}
    int status() const { return status_; }
    const kme_epoch_status& epoch_status() const { return st_; }

private:
    int status_;
    kme_epoch_status st_;
};

class MatchingEngine {
public:
    MatchingEngine(const kme_config& cfg, uint32_t epoch_records);
    ~MatchingEngine();
    MatchingEngine(const MatchingEngine&) = delete;
    MatchingEngine& operator=(const MatchingEngine&) = delete;

    void init(ProcessorContext* context);
    void process(const std::string& key, const Order& order);
    void punctuate();
    void close();
    const kme_epoch_status& last_status() const { return last_; }

private:
    void flush();
    void forward_range(uint32_t n);   // the reference's records of buffered inputs [0, n)

    kme_config cfg_;
    uint32_t epoch_records_;
    kme_engine* engine_ = nullptr;
    ProcessorContext* context_ = nullptr;
    bool dead_ = false;
    int64_t stream_base_ = 0;
    kme_epoch_status last_{};
    // pending epoch (SoA) and result buffers
    std::vector<int32_t> action_, price_, size_;
    std::vector<int64_t> oid_, aid_, sid_;
    std::vector<int32_t> out_action_, out_size_;
    std::vector<int64_t> out_prev_;
    std::vector<uint8_t> out_flags_;
    std::vector<uint32_t> trade_off_;
    std::vector<kme_trade> trades_;
};

}  // namespace kme
