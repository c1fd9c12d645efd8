// GeoHipPointPolygonRangeQuery.java -- drop-in for PointPolygonRangeQuery (same constructor and run
// signature, PointPolygonRangeQuery.java:26-30): the G / C cell filter and the per-cell window body
// with JTS point.distance(polygon) (PointPolygonRangeQuery.java:76-124, RealTime :33-73) become one
// geohip_range_ppoly call per window with the query polygon's rings (shell and holes as
// Polygon(List<List<Coordinate>>) built them); the very Point objects are emitted.  Source only
// here; built by jvm/build.sh.
package GeoFlink.spatialOperators.geohip;

import GeoFlink.spatialIndices.SpatialIndex;
import GeoFlink.spatialIndices.UniformGrid;
import GeoFlink.spatialObjects.Point;
import GeoFlink.spatialObjects.Polygon;
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
import java.util.Collections;
import java.util.List;

public class GeoHipPointPolygonRangeQuery extends RangeQuery<Point, Polygon> {
    public GeoHipPointPolygonRangeQuery(QueryConfiguration conf, SpatialIndex index) {
        super.initializeRangeQuery(conf, index);
    }

    public DataStream<Point> run(DataStream<Point> pointStream, Polygon queryPolygon, double queryRadius) {
        final QueryConfiguration conf = this.getQueryConfiguration();
        final boolean approximate = conf.isApproximateQuery();
        final double[] grid = GeoHip.grid((UniformGrid) this.getSpatialIndex());
        final List<Double> lx = new ArrayList<>(), ly = new ArrayList<>();
        final int[][] rings = GeoHip.rings(Collections.singletonList(queryPolygon), lx, ly);
        final double[] vx = GeoHip.unbox(lx), vy = GeoHip.unbox(ly);
        return pointStream.windowAll(GeoHipWindows.rangeWindows(conf))
                .apply(new RichAllWindowFunction<Point, Point, TimeWindow>() {
                    private transient GeoHip hip;

                    @Override
                    public void open(Configuration c) { hip = GeoHipWindows.open(); }

                    @Override
                    public void close() { if (hip != null) hip.close(); }

                    @Override
                    public void apply(TimeWindow w, Iterable<Point> pts, Collector<Point> out) {
                        List<Point> win = new ArrayList<>();
                        pts.forEach(win::add);
                        ByteBuffer[] xy = GeoHip.coords(win);
                        int[] pairs = hip.rangePPoly(grid, xy[0], xy[1], win.size(), rings[0], rings[1], vx, vy,
                                                     queryRadius, approximate);
                        for (int j = 0; j + 1 < pairs.length; j += 2) out.collect(win.get(pairs[j + 1]));
                    }
                });
    }
}
