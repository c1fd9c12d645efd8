// GeoHipPointPointJoinQuery.java -- drop-in for PointPointJoinQuery (same constructor and run
// signature, PointPointJoinQuery.java:20-24): the query stream's replication to its neighbouring
// cells (JoinQuery.getReplicatedPointQueryStream, JoinQuery.java:73-90) and the keyed window join
// with its distance filter (PointPointJoinQuery.java:113-172, RealTime :41-105) become one
// geohip_join_pp call per window over both streams' window contents (co-grouped on one key); each
// pair is emitted as Tuple2(ordinary point, query point), the very objects received.  Source only
// here; built by jvm/build.sh.
package GeoFlink.spatialOperators.geohip;

import GeoFlink.spatialIndices.SpatialIndex;
import GeoFlink.spatialIndices.UniformGrid;
import GeoFlink.spatialObjects.Point;
import GeoFlink.spatialOperators.QueryConfiguration;
import GeoFlink.spatialOperators.join.JoinQuery;
import GeoFlink.utils.GeoHip;
import org.apache.flink.api.common.functions.RichCoGroupFunction;
import org.apache.flink.api.java.functions.KeySelector;
import org.apache.flink.api.java.tuple.Tuple2;
import org.apache.flink.configuration.Configuration;
import org.apache.flink.streaming.api.datastream.DataStream;
import org.apache.flink.util.Collector;

import java.nio.ByteBuffer;
import java.util.ArrayList;
import java.util.List;

public class GeoHipPointPointJoinQuery extends JoinQuery<Point, Point> {
    public GeoHipPointPointJoinQuery(QueryConfiguration conf, SpatialIndex index1, SpatialIndex index2) {
        super.initializeJoinQuery(conf, index1, index2);
    }

    /** Every element on one key: a window's two sides meet in one coGroup call. */
    static final class OneKey implements KeySelector<Point, Integer> {
        @Override
        public Integer getKey(Point p) { return 0; }
    }

    public DataStream<Tuple2<Point, Point>> run(DataStream<Point> ordinaryPointStream, DataStream<Point> queryPointStream,
                                                double queryRadius) {
        final QueryConfiguration conf = this.getQueryConfiguration();
        final boolean approximate = conf.isApproximateQuery();
        final double[] uGrid = GeoHip.grid((UniformGrid) this.getSpatialIndex1());
        final double[] qGrid = GeoHip.grid((UniformGrid) this.getSpatialIndex2());
        return GeoHipWindows.withTimestamps(ordinaryPointStream, conf)
                .coGroup(GeoHipWindows.withTimestamps(queryPointStream, conf))
                .where(new OneKey()).equalTo(new OneKey())
                .window(GeoHipWindows.windows(conf))
                .apply(new RichCoGroupFunction<Point, Point, Tuple2<Point, Point>>() {
                    private transient GeoHip hip;

                    @Override
                    public void open(Configuration c) { hip = GeoHipWindows.open(); }

                    @Override
                    public void close() { if (hip != null) hip.close(); }

                    @Override
                    public void coGroup(Iterable<Point> ordinary, Iterable<Point> query, Collector<Tuple2<Point, Point>> out) {
                        List<Point> data = new ArrayList<>(), queries = new ArrayList<>();
                        ordinary.forEach(data::add);
                        query.forEach(queries::add);
                        if (data.isEmpty() || queries.isEmpty()) return;
                        ByteBuffer[] d = GeoHip.coords(data), q = GeoHip.coords(queries);
                        int[] pairs = hip.joinPP(uGrid, qGrid, d[0], d[1], data.size(), q[0], q[1], queries.size(),
                                                 queryRadius, approximate);
                        for (int j = 0; j + 1 < pairs.length; j += 2)
                            out.collect(Tuple2.of(data.get(pairs[j]), queries.get(pairs[j + 1])));
                    }
                });
    }
}
