// TEST INFRASTRUCTURE ONLY.  Driver that links the *reference's own* PID header
// (/root/reference/include/fast_kinematic_simulator/simple_pid_controller.hpp,
// std-only) to emit golden vectors for the PID restatement.
// Built by `make -C oracle ref` into oracle/_ref/ (git-ignored); the reference
// source is compiled where it lies, never copied.
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fast_kinematic_simulator/simple_pid_controller.hpp>

// `pid_golden --replay`: reads "kp ki kd iclamp n" then n lines "error dt" (C99 hex
// floats) from stdin and prints one hex-float ComputeFeedbackTerm output per line, from
// a fresh controller (Zero() state).  Used by tests/golden/make_pid_trace_golden.py to
// run error sequences taken from a simulation trace through the reference's PID.
static int replay() {
    double kp, ki, kd, iclamp;
    long n = 0;
    while (std::scanf("%la %la %la %la %ld", &kp, &ki, &kd, &iclamp, &n) == 5) {
        simple_pid_controller::SimplePIDController pid(kp, ki, kd, iclamp);
        for (long i = 0; i < n; ++i) {
            double e, dt;
            if (std::scanf("%la %la", &e, &dt) != 2) return 1;
            std::printf("%a\n", pid.ComputeFeedbackTerm(e, dt));
        }
    }
    return 0;
}

int main(int argc, char** argv) {
    if (argc > 1 && std::strcmp(argv[1], "--replay") == 0) return replay();
    // cases: kp, ki, kd, iclamp (negative gains exercise Initialize()'s abs)
    const double cases[][4] = {{1.0, 0.1, 0.01, 1.0}, {10.0, 1.0, 0.1, 0.5}, {-2.0, -0.5, -0.2, -0.25}, {4.0, 0.0, 0.0, 0.0}};
    std::printf("{\n  \"source\": \"reference simple_pid_controller.hpp via oracle/ref/pid_golden_driver.cpp\",\n  \"cases\": [\n");
    unsigned long long s = 88172645463325252ull;
    for (int c = 0; c < 4; ++c) {
        simple_pid_controller::SimplePIDController pid(cases[c][0], cases[c][1], cases[c][2], cases[c][3]);
        std::printf("    {\"kp\": %.17g, \"ki\": %.17g, \"kd\": %.17g, \"iclamp\": %.17g, \"steps\": [", cases[c][0], cases[c][1],
                    cases[c][2], cases[c][3]);
        for (int i = 0; i < 64; ++i) {
            s ^= s << 13; s ^= s >> 7; s ^= s << 17;
            const double e = ((double)(s >> 11) / 9007199254740992.0 - 0.5) * 4.0;
            s ^= s << 13; s ^= s >> 7; s ^= s << 17;
            const double dt = (i % 3 == 0) ? 0.01 : ((double)(s >> 11) / 9007199254740992.0) * 0.05 + 0.001;
            if (i == 20) pid.Zero();
            const double out = pid.ComputeFeedbackTerm(e, dt);
            std::printf("%s[%.17g, %.17g, %.17g, %d]", i ? ", " : "", e, dt, out, i == 20 ? 1 : 0);
        }
        std::printf("]}%s\n", c < 3 ? "," : "");
    }
    std::printf("  ]\n}\n");
    return 0;
}
