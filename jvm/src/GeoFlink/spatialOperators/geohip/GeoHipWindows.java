// GeoHipWindows.java -- the window assigners and the per-task-thread libgeohip context shared by
// the drop-in operators of this package.  Source only here (no JDK in this image); jvm/build.sh.
//
// Window semantics stay the reference's (SURVEY.md 8(a) a16): WindowBased queries evaluate the
// contents of each SlidingProcessingTimeWindows(size, slide) window
// (PointPointRangeQuery.java:116, PointPointKNNQuery.java:151/189, PointPointJoinQuery.java:148,
// PointPolygonRangeQuery.java:103); RealTime range queries are per-record predicates, evaluated here
// over short processing-time micro-batches with the identical predicate; RealTime kNN / join use the
// reference's TumblingEventTimeWindows(windowSize) over timestamps with bounded out-of-orderness
// (PointPointKNNQuery.java:58-122, PointPointJoinQuery.java:41-105).  The difference from the
// reference is only where a window is evaluated: one native call per window instead of one
// keyBy(gridID) group per cell.
package GeoFlink.spatialOperators.geohip;

import GeoFlink.spatialObjects.SpatialObject;
import GeoFlink.spatialOperators.QueryConfiguration;
import GeoFlink.spatialOperators.QueryType;
import GeoFlink.utils.GeoHip;
import org.apache.flink.streaming.api.datastream.DataStream;
import org.apache.flink.streaming.api.functions.timestamps.BoundedOutOfOrdernessTimestampExtractor;
import org.apache.flink.streaming.api.windowing.assigners.SlidingProcessingTimeWindows;
import org.apache.flink.streaming.api.windowing.assigners.TumblingEventTimeWindows;
import org.apache.flink.streaming.api.windowing.assigners.TumblingProcessingTimeWindows;
import org.apache.flink.streaming.api.windowing.assigners.WindowAssigner;
import org.apache.flink.streaming.api.windowing.time.Time;
import org.apache.flink.streaming.api.windowing.windows.TimeWindow;

final class GeoHipWindows {
    private GeoHipWindows() {}

    /** HIP device of this JVM's contexts (GEOHIP_DEVICE, default 0). */
    static int device() {
        String d = System.getenv("GEOHIP_DEVICE");
        return d == null ? 0 : Integer.parseInt(d);
    }

    /** Milliseconds of a RealTime range micro-batch (GEOHIP_REALTIME_BATCH_MS, default 100). */
    static long realTimeBatchMs() {
        String d = System.getenv("GEOHIP_REALTIME_BATCH_MS");
        return d == null ? 100L : Long.parseLong(d);
    }

    static GeoHip open() { return new GeoHip(device()); }

    /** The window of a range query: the reference's sliding processing-time window, or RealTime
     *  micro-batches. */
    static WindowAssigner<Object, TimeWindow> rangeWindows(QueryConfiguration conf) {
        if (conf.getQueryType() == QueryType.RealTime)
            return TumblingProcessingTimeWindows.of(Time.milliseconds(realTimeBatchMs()));
        if (conf.getQueryType() == QueryType.WindowBased)
            return SlidingProcessingTimeWindows.of(Time.seconds(conf.getWindowSize()), Time.seconds(conf.getSlideStep()));
        throw new IllegalArgumentException("Not yet support");
    }

    /** The window of a kNN or join query: the reference's sliding processing-time window, or its
     *  RealTime tumbling event-time window of windowSize seconds. */
    static WindowAssigner<Object, TimeWindow> windows(QueryConfiguration conf) {
        if (conf.getQueryType() == QueryType.RealTime)
            return TumblingEventTimeWindows.of(Time.seconds(conf.getWindowSize()));
        if (conf.getQueryType() == QueryType.WindowBased)
            return SlidingProcessingTimeWindows.of(Time.seconds(conf.getWindowSize()), Time.seconds(conf.getSlideStep()));
        throw new IllegalArgumentException("Not yet support");
    }

    /** RealTime event-time windows need the reference's timestamps and watermarks
     *  (objects' timeStampMillisec, bounded out-of-orderness of allowedLateness seconds). */
    static <T extends SpatialObject> DataStream<T> withTimestamps(DataStream<T> s, QueryConfiguration conf) {
        if (conf.getQueryType() != QueryType.RealTime) return s;
        return s.assignTimestampsAndWatermarks(
                new BoundedOutOfOrdernessTimestampExtractor<T>(Time.seconds(conf.getAllowedLateness())) {
                    @Override
                    public long extractTimestamp(T o) { return o.timeStampMillisec; }
                });
    }
}
