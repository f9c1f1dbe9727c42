/* Mock ROS message (test only; tests/cpp/mock_workspace/README.md) */
#ifndef MOCK_STD_MSGS_COLORRGBA
#define MOCK_STD_MSGS_COLORRGBA
#include <string>
namespace std_msgs {
struct ColorRGBA {
    float r = 0.0f, g = 0.0f, b = 0.0f, a = 0.0f;
};
struct Header {
    unsigned int seq = 0;
    std::string frame_id;
};
}  // namespace std_msgs
#endif
