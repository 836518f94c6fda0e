/*
 * kme_processor.h -- C ABI of the host-side mirror of the reference's stream processor.
 *
 * The reference plugs `MatchingEngine implements Processor<String, Order>` into its topology
 * (/root/reference/src/main/java/KProcessor.java:52, 63-129): init(ProcessorContext),
 * process(String key, Order value) once per record, close(); the context forwards (key, Order)
 * to the MatchOut sink, which serialises with Jackson (KP:477-495).
 *
 * kme_processor keeps that contract over the epoch engine of kme.h: process() takes one JSON
 * record (the MatchIn value), records are batched into epochs of `epoch_records`, and at each
 * flush (epoch full, punctuate, close) the forward callback receives, in reference order, every
 * record the reference would have forwarded: ("IN", value), fills ("OUT", ...), ("OUT", value),
 * as the exact bytes JsonSerializer would have produced.  commit() is requested once per epoch.
 * This is the JNI/FFM-facing shape; INTEGRATION.md shows the Java side.
 */
#ifndef KME_PROCESSOR_H
#define KME_PROCESSOR_H
#include <stddef.h>
#include <stdint.h>

#include "kme.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef void (*kme_forward_fn)(void* user, const char* key, const char* value, size_t value_len);
typedef void (*kme_commit_fn)(void* user);

typedef struct kme_processor kme_processor;

/* MatchingEngine::new + init(context) (KP:52, 86-93). */
kme_status kme_processor_create(const kme_config* cfg, uint32_t epoch_records, kme_forward_fn forward,
                                kme_commit_fn commit, void* user, kme_processor** out);
/* process(key, value) (KP:96): `json` is the MatchIn value bytes; the key is ignored as in KP:96.
 * Returns KME_E_INVALID for bytes JsonDeserializer would reject (a SerializationException). */
kme_status kme_processor_process_json(kme_processor* p, const char* json, size_t len);
/* Same, already decoded. */
kme_status kme_processor_process(kme_processor* p, int32_t action, int64_t oid, int64_t aid, int64_t sid,
                                 int32_t price, int32_t size);
/* Punctuator: flush the pending epoch now (wall-clock punctuation in the Java shim). */
kme_status kme_processor_punctuate(kme_processor* p);
/* close() (KP:129): flushes, then releases the engine. */
kme_status kme_processor_close(kme_processor* p);
/* Status of the last flush (error index is relative to the stream). */
kme_status kme_processor_last_status(kme_processor* p, kme_epoch_status* st);

#ifdef __cplusplus
}
#endif
#endif
