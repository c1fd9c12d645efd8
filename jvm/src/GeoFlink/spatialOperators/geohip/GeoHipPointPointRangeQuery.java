// GeoHipPointPointRangeQuery.java -- drop-in for PointPointRangeQuery (same constructor and run
// signature, PointPointRangeQuery.java:32-36): the per-cell filter + keyBy(gridID) + window body
// (PointPointRangeQuery.java:86-137, RealTime :43-83) becomes one geohip_range_pp call per window
// that returns the positions of the qualifying points; the very Point objects are emitted.
// Source only here (no JDK in this image); built by jvm/build.sh.
package GeoFlink.spatialOperators.geohip;

import GeoFlink.spatialIndices.SpatialIndex;
import GeoFlink.spatialIndices.UniformGrid;
import GeoFlink.spatialObjects.Point;
import GeoFlink.spatialOperators.QueryConfiguration;
import GeoFlink.spatialOperators.range.RangeQuery;
import GeoFlink.utils.GeoHip;
import org.apache.flink.configuration.Configuration;
import org.apache.flink.streaming.api.datastream.DataStream;
import org.apache.flink.streaming.api.functions.windowing.RichAllWindowFunction;
import org.apache.flink.streaming.api.windowing.windows.TimeWindow;
import org.apache.flink.util.Collector;

import java.nio.ByteBuffer;
import java.util.ArrayList;
import java.util.List;

public class GeoHipPointPointRangeQuery extends RangeQuery<Point, Point> {
    public GeoHipPointPointRangeQuery(QueryConfiguration conf, SpatialIndex index) {
        super.initializeRangeQuery(conf, index);
    }

    public DataStream<Point> run(DataStream<Point> pointStream, Point queryPoint, double queryRadius) {
        final QueryConfiguration conf = this.getQueryConfiguration();
        final boolean approximate = conf.isApproximateQuery();
        final double[] grid = GeoHip.grid((UniformGrid) this.getSpatialIndex());
        final double qx = queryPoint.point.getX(), qy = queryPoint.point.getY();
        return pointStream.windowAll(GeoHipWindows.rangeWindows(conf))
                .apply(new RichAllWindowFunction<Point, Point, TimeWindow>() {
                    private transient GeoHip hip;  // one libgeohip context per task thread

                    @Override
                    public void open(Configuration c) { hip = GeoHipWindows.open(); }

                    @Override
                    public void close() { if (hip != null) hip.close(); }

                    @Override
                    public void apply(TimeWindow w, Iterable<Point> pts, Collector<Point> out) {
                        List<Point> win = new ArrayList<>();
                        pts.forEach(win::add);
                        ByteBuffer[] xy = GeoHip.coords(win);
                        for (int i : hip.rangePP(grid, xy[0], xy[1], win.size(), qx, qy, queryRadius, approximate))
                            out.collect(win.get(i));
                    }
                });
    }
}
