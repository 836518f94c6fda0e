// GpuMatchingEngine -- the MI355X matching engine behind the reference's Processor interface, the
// one-line swap at the topology (KProcessor.java:52):
//
//     .addProcessor("MatchingEngine", GpuMatchingEngine::new, "Source")
//
// Contract kept from MatchingEngine (KP:96-126): for every input record the processor forwards
// ("IN", order), then the maker and the taker fill of each trade (keyed "OUT", KP:272-273), then
// ("OUT", order) -- same order, same field values.  The difference is timing: records are buffered
// into an epoch and forwarded when the epoch is flushed (full, or at the wall-clock punctuation),
// and the offset commit is requested after the flush.  On a fault the records before it are
// forwarded and committed (as the reference's per-record commit would have, KP:97, 124-125) and
// the processor then fails like the reference's stream thread; KME_E_UNFUNDED (FUNDED mode
// without KME_FLAG_SERIAL_FALLBACK) refuses the records from the unprovable one on without
// changing anything -- they stay buffered and are retried at the next flush.
//
// Native side: kme_jni.c (libkme_jni.so, linked against libkme.so).  The record type is the
// reference's KProcessor.Order (KP:448-476); this file only uses its public fields and
// constructor.
import java.time.Duration;

import org.apache.kafka.streams.processor.Processor;
import org.apache.kafka.streams.processor.ProcessorContext;
import org.apache.kafka.streams.processor.PunctuationType;

public final class GpuMatchingEngine implements Processor<String, KProcessor.Order> {
    static { System.loadLibrary("kme_jni"); }

    // include/kme.h
    static final int KME_MODE_EXACT = 0, KME_MODE_FUNDED = 1;
    static final int KME_FLAG_EXACT_LEDGER = 1, KME_FLAG_SERIAL_FALLBACK = 2;
    static final int KME_OK = 0, KME_E_UNFUNDED = 4;

    private static native long create(int mode, int maxSymbols, int maxEpoch, long maxResting, int maxTrades,
                                      int maxAccounts, int flags, int device);
    private static native void destroy(long h);
    private static native int submit(long h, int n, int[] action, long[] oid, long[] aid, long[] sid, int[] price,
                                     int[] size, byte[] kind, int[] oAction, long[] oOid, long[] oAid, long[] oSid,
                                     int[] oPrice, int[] oSize, long[] oPrev, byte[] oHasPrev, long[] status);
    private static native String statusText(int status);
    static native int checkpoint(long h, String path);
    static native int restore(long h, String path);

    private final int epoch;
    private final int maxTrades;
    private ProcessorContext context;
    private long h;
    private int n;
    private final int[] action, price, size;
    private final long[] oid, aid, sid;
    private final byte[] kind, oHasPrev;
    private final int[] oAction, oPrice, oSize;
    private final long[] oOid, oAid, oSid, oPrev;
    private final long[] status = new long[3];

    public GpuMatchingEngine() { this(1 << 16, 1 << 18); }

    public GpuMatchingEngine(int epoch, int maxTrades) {
        this.epoch = epoch;
        this.maxTrades = maxTrades;
        action = new int[epoch]; price = new int[epoch]; size = new int[epoch];
        oid = new long[epoch]; aid = new long[epoch]; sid = new long[epoch];
        final int rows = 2 * epoch + 2 * maxTrades;   // IN + OUT per record, two fills per trade
        kind = new byte[rows]; oHasPrev = new byte[rows];
        oAction = new int[rows]; oPrice = new int[rows]; oSize = new int[rows];
        oOid = new long[rows]; oAid = new long[rows]; oSid = new long[rows]; oPrev = new long[rows];
    }

    @Override public void init(ProcessorContext context) {             // KP:86-93
        this.context = context;
        // EXACT reproduces every store (one wavefront, arrival order); FUNDED runs symbols in
        // parallel, with the exact ledger kept and serial fallback for unprovable epochs
        this.h = create(KME_MODE_FUNDED, 1 << 16, epoch, 1L << 26, maxTrades, 1 << 20,
                        KME_FLAG_EXACT_LEDGER | KME_FLAG_SERIAL_FALLBACK, 0);
        context.schedule(Duration.ofMillis(1), PunctuationType.WALL_CLOCK_TIME, ts -> flush());
    }

    @Override public void process(String key, KProcessor.Order o) {      // KP:96
        action[n] = o.action; oid[n] = o.oid; aid[n] = o.aid; sid[n] = o.sid;
        price[n] = o.price; size[n] = o.size;
        if (++n == epoch) flush();
    }

    private void flush() {
        if (n == 0) return;
        final int rows = submit(h, n, action, oid, aid, sid, price, size,
                                kind, oAction, oOid, oAid, oSid, oPrice, oSize, oPrev, oHasPrev, status);
        for (int k = 0; k < rows; k++) {
            KProcessor.Order r = new KProcessor.Order(oAction[k], oOid[k], oAid[k], oSid[k], oPrice[k], oSize[k]);
            if (kind[k] == 2 && oHasPrev[k] != 0) r.prev = oPrev[k];     // OUT echo of addOrder (KP:218)
            context.forward(kind[k] == 0 ? "IN" : "OUT", r);
        }
        final int s = (int) status[0];
        if (s == KME_OK) {
            n = 0;
            context.commit();
            return;
        }
        // the records before the one at status[2] took effect and were forwarded: commit them
        final int done = status[2] < 0 ? 0 : (int) status[2];
        System.arraycopy(action, done, action, 0, n - done);
        System.arraycopy(oid, done, oid, 0, n - done);
        System.arraycopy(aid, done, aid, 0, n - done);
        System.arraycopy(sid, done, sid, 0, n - done);
        System.arraycopy(price, done, price, 0, n - done);
        System.arraycopy(size, done, size, 0, n - done);
        n -= done;
        context.commit();
        if (s != KME_E_UNFUNDED) throw new IllegalStateException(statusText(s));   // the stream thread dies
    }

    @Override public void close() {                                     // KP:129
        flush();
        destroy(h);
    }
}
