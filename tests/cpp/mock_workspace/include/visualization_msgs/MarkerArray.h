/* Mock ROS messages (test only; tests/cpp/mock_workspace/README.md): the fields the
 * reference's display helpers set (SPCS:612-646, 725-735) */
#ifndef MOCK_VISUALIZATION_MSGS_MARKERARRAY
#define MOCK_VISUALIZATION_MSGS_MARKERARRAY
#include <cstdint>
#include <string>
#include <vector>
#include <geometry_msgs/Point.h>
#include <std_msgs/ColorRGBA.h>
namespace visualization_msgs {
struct Marker {
    enum { ARROW = 0u, CUBE = 1u, SPHERE = 2u, CYLINDER = 3u, LINE_STRIP = 4u, LINE_LIST = 5u, CUBE_LIST = 6u, SPHERE_LIST = 7u };
    enum { ADD = 0u, MODIFY = 0u, DELETE = 2u };
    std_msgs::Header header;
    std::string ns;
    int32_t id = 0;
    int32_t type = 0;
    int32_t action = 0;
    geometry_msgs::Vector3 scale;
    std_msgs::ColorRGBA color;
    bool frame_locked = false;
    std::vector<geometry_msgs::Point> points;
    std::vector<std_msgs::ColorRGBA> colors;
};
struct MarkerArray {
    std::vector<Marker> markers;
};
}  // namespace visualization_msgs
#endif
