// GeoHipPointPointKNNQuery.java -- drop-in for PointPointKNNQuery (same constructor and run
// signature, PointPointKNNQuery.java:29-33): the per-cell heaps (PointPointKNNQuery.java:125-182,
// RealTime :58-122) and the parallelism-1 windowAll merge (KNNQuery.java:204-272) become one
// geohip_knn_pp call per window.  The emitted Tuple3(window start, window end, PriorityQueue) holds
// the k nearest of the window's G u C points in the reference's heap type and comparator; the
// library's order is ascending (distance, window position), without the merge bug of
// KNNQuery.java:249-251 (SURVEY.md appendix 5).  Source only here; built by jvm/build.sh.
package GeoFlink.spatialOperators.geohip;

import GeoFlink.spatialIndices.SpatialIndex;
import GeoFlink.spatialIndices.UniformGrid;
import GeoFlink.spatialObjects.Point;
import GeoFlink.spatialOperators.QueryConfiguration;
import GeoFlink.spatialOperators.knn.KNNQuery;
import GeoFlink.utils.Comparators;
import GeoFlink.utils.GeoHip;
import org.apache.flink.api.java.tuple.Tuple2;
import org.apache.flink.api.java.tuple.Tuple3;
import org.apache.flink.configuration.Configuration;
import org.apache.flink.streaming.api.datastream.DataStream;
import org.apache.flink.streaming.api.functions.windowing.RichAllWindowFunction;
import org.apache.flink.streaming.api.windowing.windows.TimeWindow;
import org.apache.flink.util.Collector;

import java.nio.ByteBuffer;
import java.util.ArrayList;
import java.util.List;
import java.util.PriorityQueue;

public class GeoHipPointPointKNNQuery extends KNNQuery<Point, Point> {
    public GeoHipPointPointKNNQuery(QueryConfiguration conf, SpatialIndex index) {
        super.initializeKNNQuery(conf, index);
    }

    public DataStream<Tuple3<Long, Long, PriorityQueue<Tuple2<Point, Double>>>> run(DataStream<Point> pointStream,
                                                                                   Point queryPoint, double queryRadius,
                                                                                   Integer k) {
        final QueryConfiguration conf = this.getQueryConfiguration();
        final double[] grid = GeoHip.grid((UniformGrid) this.getSpatialIndex());
        final double qx = queryPoint.point.getX(), qy = queryPoint.point.getY();
        final int kk = k;
        return GeoHipWindows.withTimestamps(pointStream, conf).windowAll(GeoHipWindows.windows(conf))
                .apply(new RichAllWindowFunction<Point, Tuple3<Long, Long, PriorityQueue<Tuple2<Point, Double>>>, TimeWindow>() {
                    private transient GeoHip hip;

                    @Override
                    public void open(Configuration c) { hip = GeoHipWindows.open(); }

                    @Override
                    public void close() { if (hip != null) hip.close(); }

                    @Override
                    public void apply(TimeWindow w, Iterable<Point> pts,
                                      Collector<Tuple3<Long, Long, PriorityQueue<Tuple2<Point, Double>>>> out) {
                        List<Point> win = new ArrayList<>();
                        pts.forEach(win::add);
                        ByteBuffer[] xy = GeoHip.coords(win);
                        int[] idx = new int[kk];
                        double[] dist = new double[kk];
                        int m = hip.knnPP(grid, xy[0], xy[1], win.size(), qx, qy, queryRadius, kk, idx, dist);
                        PriorityQueue<Tuple2<Point, Double>> q =
                                new PriorityQueue<>(Math.max(kk, 1), new Comparators.inTuplePointDistanceComparator());
                        for (int j = 0; j < m; j++) q.offer(Tuple2.of(win.get(idx[j]), dist[j]));
                        out.collect(Tuple3.of(w.getStart(), w.getEnd(), q));
                    }
                });
    }
}
