/* Mock ROS messages (test only; tests/cpp/mock_workspace/README.md) */
#ifndef MOCK_GEOMETRY_MSGS_POINT
#define MOCK_GEOMETRY_MSGS_POINT
namespace geometry_msgs {
struct Point {
    double x = 0.0, y = 0.0, z = 0.0;
};
struct Vector3 {
    double x = 0.0, y = 0.0, z = 0.0;
};
}  // namespace geometry_msgs
#endif
