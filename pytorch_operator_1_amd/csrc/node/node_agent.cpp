// pto-node-agent: the native node daemon of the single-node MI355X
// PyTorchJob stack.  It replaces the pieces of the reference's substrate
// that sit on the submit -> first-step critical path:
//
//   * kubelet process supervision: fork/exec of container processes into
//     their own process group, stdout/stderr captured to a per-container
//     log, kubelet restart semantics (Always / OnFailure / Never,
//     restartCount, exponential restart back-off = CrashLoopBackOff),
//     exit codes (128+signal for signalled deaths, as the container runtime
//     reports them), graceful kill (SIGTERM, then SIGKILL after a grace
//     period) of the whole process group;
//   * device plugin: an exclusive amd.com/gpu allocator with all-or-nothing
//     (gang) admission and per-GPU HBM accounting sized for 288 GB/GPU,
//     GPU discovery from the KFD topology, CPU affinity per allocation;
//   * the worker init-container gate: a TCP connect probe of
//     MASTER_ADDR:MASTER_PORT (the DNS wait of the reference's
//     init-pytorch container, pkg/common/config/config.go:9-20);
//   * restart groups (gang restart): the containers of one multi-replica
//     job share a group.  A DDP world cannot take back one restarted rank
//     (its peers hold the old rendezvous store and communicators), so when a
//     member fails and its policy restarts it, the agent SIGKILLs every other
//     running member, holds them all until the last one has been reaped (the
//     old rendezvous port is then closed), and restarts the whole group at
//     once with PTO_RESTART_GENERATION=<base>.<wave> -- one rendezvous per
//     wave, never a new rank joining an old store;
//   * warm starts (--zygote PYTHON): a pre-imported interpreter
//     (node/zygote.py) forks `python -m MODULE` / `python SCRIPT.py`
//     containers instead of a cold fork/exec (import torch is ~1.5-2 s of
//     the submit -> first-step path).  The agent is a child subreaper, so
//     zygote-forked containers are re-parented to it and reaped, restarted
//     and killed exactly like exec'ed ones; any other argv, or a zygote
//     that is not ready/alive, takes the fork/exec path.
//
// Protocol: one JSON object per line on a Unix socket (--socket) or on
// stdin/stdout (--stdio); every request gets exactly one JSON reply line.
// Ops: ping, spawn, kill, remove, status, gpus, alloc, free, probe, shutdown.
#include <arpa/inet.h>
#include <dirent.h>
#include <errno.h>
#include <fcntl.h>
#include <netdb.h>
#include <netinet/in.h>
#include <poll.h>
#include <sched.h>
#include <limits.h>
#include <signal.h>
#include <stdlib.h>
#include <sys/prctl.h>
#include <sys/signalfd.h>
#include <sys/socket.h>
#include <sys/stat.h>
#include <sys/types.h>
#include <sys/un.h>
#include <sys/wait.h>
#include <time.h>
#include <unistd.h>

#include <algorithm>
#include <cstdio>
#include <cstring>
#include <fstream>
#include <iostream>
#include <map>
#include <set>
#include <string>
#include <vector>

#include "json.hpp"

using pto::Json;

static double now_s() {
  timespec ts;
  clock_gettime(CLOCK_REALTIME, &ts);
  return ts.tv_sec + ts.tv_nsec * 1e-9;
}
static double mono_s() {
  timespec ts;
  clock_gettime(CLOCK_MONOTONIC, &ts);
  return ts.tv_sec + ts.tv_nsec * 1e-9;
}

// ------------------------------------------------------------------ procs --
struct Proc {
  std::string id;
  std::vector<std::string> argv;
  std::map<std::string, std::string> env;
  std::string cwd, log;
  std::string restart_policy = "Never";  // Always | OnFailure | Never
  std::vector<int> cpus;
  pid_t pid = -1;
  int restart_count = 0;
  std::string state = "waiting";  // waiting | running | terminated
  std::string reason = "ContainerCreating";
  int exit_code = 0, signal = 0;
  double started_at = 0, finished_at = 0;
  double restart_at = 0;   // monotonic time of the next (re)start
  double kill_deadline = 0;  // monotonic; SIGKILL after this
  bool stopping = false;     // killed on purpose: no restart
  int last_exit_code = 0;
  double last_finished_at = 0;
  std::string launcher;  // "zygote" | "exec"
  bool exec_only = false;  // spawn request "launcher": "exec" -- never fork from the zygote
  std::string group;       // restart group ("" = restarts alone)
  std::string gen_base;    // PTO_RESTART_GENERATION given at spawn
  bool held = false;       // restart owed, waiting for its group to drain
  double held_delay = 0;   // its own CrashLoopBackOff delay
  bool wave_killed = false;  // stopped by a group wave it did not cause: not its own restart
};

// One restart wave at a time per group: `draining` from the first failing
// member until every member has exited, then all held members restart.
struct Group {
  int wave = 0;
  bool draining = false;
  double drain_started = 0;
};

// ---------------------------------------------------------------- zygote --
struct Zygote {
  std::string python, module = "pytorch_operator_1_amd.node.zygote", pypath;
  bool spare = false;  // a warm SPARE: runs one container itself instead of forking it
  pid_t pid = -1;
  int fd = -1;
  bool ready = false;
  std::string inbuf;
  long long spawned = 0, fallbacks = 0;

  bool enabled() const { return !python.empty(); }

  void start() {
    if (python.empty()) return;
    int sv[2];
    if (socketpair(AF_UNIX, SOCK_STREAM | SOCK_CLOEXEC, 0, sv) != 0) return;
    pid_t c = fork();
    if (c == 0) {
      close(sv[0]);
      int fd = dup(sv[1]);  // no CLOEXEC: inherited by the interpreter
      sigset_t none;
      sigemptyset(&none);
      sigprocmask(SIG_SETMASK, &none, nullptr);
      int devnull = open("/dev/null", O_RDWR);
      if (devnull >= 0) {
        dup2(devnull, 0);
        dup2(devnull, 1);
        if (devnull > 2) close(devnull);
      }
      std::string pp = pypath;
      const char* old = getenv("PYTHONPATH");
      if (old && *old) pp = pp.empty() ? std::string(old) : pp + ":" + old;
      if (!pp.empty()) setenv("PYTHONPATH", pp.c_str(), 1);
      std::string fds = std::to_string(fd);
      if (spare)
        execlp(python.c_str(), python.c_str(), "-m", module.c_str(), "--fd", fds.c_str(), "--spare", (char*)nullptr);
      else
        execlp(python.c_str(), python.c_str(), "-m", module.c_str(), "--fd", fds.c_str(), (char*)nullptr);
      _exit(127);
    }
    close(sv[1]);
    if (c < 0) {
      close(sv[0]);
      return;
    }
    pid = c;
    fd = sv[0];
    ready = false;
    inbuf.clear();
  }

  void died() {
    if (fd >= 0) close(fd);
    fd = -1;
    pid = -1;
    ready = false;
  }

  // non-blocking: consume the "ready" line once the interpreter is warm
  void poll_ready() {
    if (fd < 0 || ready) return;
    char buf[4096];
    while (true) {
      ssize_t r = recv(fd, buf, sizeof buf, MSG_DONTWAIT);
      if (r > 0) {
        inbuf.append(buf, r);
        continue;
      }
      if (r == 0) {
        died();
        return;
      }
      break;
    }
    size_t nl = inbuf.find('\n');
    if (nl == std::string::npos) return;
    std::string line = inbuf.substr(0, nl);
    inbuf.erase(0, nl + 1);
    try {
      ready = Json::parse(line)["ready"].boolean(false);
    } catch (std::exception&) {
      ready = false;
    }
  }

  // python [-u] (-m MODULE | SCRIPT.py) ... of the zygote's own interpreter
  bool eligible(const std::vector<std::string>& argv) const {
    if (argv.size() < 2) return false;
    char a[PATH_MAX], b[PATH_MAX];
    if (!realpath(argv[0].c_str(), a) || !realpath(python.c_str(), b) || strcmp(a, b) != 0) return false;
    size_t i = 1;
    while (i < argv.size() && argv[i] == "-u") ++i;
    if (i >= argv.size()) return false;
    if (argv[i] == "-m") return i + 1 < argv.size();
    const std::string& s = argv[i];
    return s.size() > 3 && s.compare(s.size() - 3, 3, ".py") == 0 && s[0] != '-';
  }

  // one request, one reply line (a fork takes milliseconds); -1 on any
  // failure, and the caller falls back to fork/exec
  pid_t spawn(const Json& req) {
    if (!ready || fd < 0) return -1;
    std::string line = req.dump() + "\n";
    size_t off = 0;
    while (off < line.size()) {
      ssize_t w = send(fd, line.data() + off, line.size() - off, MSG_NOSIGNAL);
      if (w <= 0) {
        died();
        return -1;
      }
      off += (size_t)w;
    }
    const double end = mono_s() + 10.0;
    while (true) {
      size_t nl = inbuf.find('\n');
      if (nl != std::string::npos) {
        std::string l = inbuf.substr(0, nl);
        inbuf.erase(0, nl + 1);
        try {
          Json r = Json::parse(l);
          if (!r["ok"].boolean(false)) return -1;
          return (pid_t)r["pid"].num(-1);
        } catch (std::exception&) {
          return -1;
        }
      }
      double left = end - mono_s();
      if (left <= 0) {  // a late reply would desynchronise the protocol: drop this zygote
        ::kill(pid, SIGKILL);
        died();
        return -1;
      }
      pollfd pf{fd, POLLIN, 0};
      if (poll(&pf, 1, (int)(left * 1000) + 1) <= 0) continue;
      char buf[4096];
      ssize_t r = recv(fd, buf, sizeof buf, 0);
      if (r <= 0) {
        died();
        return -1;
      }
      inbuf.append(buf, r);
    }
  }
};

struct Agent {
  std::map<std::string, Proc> procs;
  std::map<std::string, Group> groups;
  // GPU allocator
  int n_gpus = 0;
  double hbm_per_gpu = 288e9;
  std::vector<std::string> gpu_owner;
  std::vector<double> gpu_hbm;
  std::vector<int> gpu_numa;
  double backoff_base = 0.2, backoff_max = 10.0;
  bool quit = false;
  Zygote zygote;
  // Warm spare for the containers that must NOT be forked from the zygote
  // (the rendezvous store host of a multi-rank job: its TCPStore server hung
  // in forked interpreters): an exec'ed interpreter that has already done the
  // zygote's imports and runs exactly one container itself -- the cold
  // `import torch` (~2.4 s on the MI355X box) is off that replica's submit ->
  // first step path.  A used spare is replaced at once.
  Zygote spare;
  long long spares_used = 0;

  void discover_gpus(int forced) {
    if (forced >= 0) {
      n_gpus = forced;
    } else {
      n_gpus = 0;
      DIR* d = opendir("/sys/class/kfd/kfd/topology/nodes");
      if (d) {
        std::vector<std::string> nodes;
        while (dirent* e = readdir(d))
          if (e->d_name[0] != '.') nodes.push_back(e->d_name);
        closedir(d);
        std::sort(nodes.begin(), nodes.end(), [](const std::string& a, const std::string& b) {
          return atoi(a.c_str()) < atoi(b.c_str());
        });
        for (auto& nd : nodes) {
          std::ifstream f("/sys/class/kfd/kfd/topology/nodes/" + nd + "/properties");
          std::string k;
          long long v;
          long long simd = 0, numa = -1;
          while (f >> k >> v) {
            if (k == "simd_count") simd = v;
            if (k == "numa_node") numa = v;  // not always present
          }
          if (simd > 0) {
            ++n_gpus;
            gpu_numa.push_back((int)numa);
          }
        }
      }
    }
    gpu_numa.resize(n_gpus, -1);
    gpu_owner.assign(n_gpus, "");
    gpu_hbm.assign(n_gpus, 0.0);
  }

  // ------------------------------------------------------------- spawn --
  bool start_zygote(Proc& p) {
    if (p.exec_only || !zygote.enabled() || !zygote.ready || !zygote.eligible(p.argv)) return false;
    Json req = Json::object();
    Json argv = Json::array();
    for (auto& a : p.argv) argv.push(a);
    req["argv"] = argv;
    Json env = Json::object();
    for (auto& kv : p.env) env[kv.first] = kv.second;
    req["env"] = env;
    req["cwd"] = p.cwd;
    req["log"] = p.log;
    Json cpus = Json::array();
    for (int c : p.cpus) cpus.push(c);
    req["cpus"] = cpus;
    pid_t pid = zygote.spawn(req);
    if (pid <= 0) {
      ++zygote.fallbacks;
      return false;
    }
    ++zygote.spawned;
    p.pid = pid;
    p.state = "running";
    p.reason = "";
    p.started_at = now_s();
    p.launcher = "zygote";
    return true;
  }

  bool start_spare(Proc& p) {
    if (!p.exec_only || !spare.enabled() || !spare.ready || !spare.eligible(p.argv)) return false;
    Json req = Json::object();
    Json argv = Json::array();
    for (auto& a : p.argv) argv.push(a);
    req["argv"] = argv;
    Json env = Json::object();
    for (auto& kv : p.env) env[kv.first] = kv.second;
    req["env"] = env;
    req["cwd"] = p.cwd;
    req["log"] = p.log;
    Json cpus = Json::array();
    for (int c : p.cpus) cpus.push(c);
    req["cpus"] = cpus;
    const pid_t sp = spare.pid;
    pid_t pid = spare.spawn(req);
    if (pid <= 0 || pid != sp) return false;  // spawn() already dropped a broken spare
    // the spare process IS the container from now on: forget it as a spare
    if (spare.fd >= 0) close(spare.fd);
    spare.fd = -1;
    spare.pid = -1;
    spare.ready = false;
    ++spares_used;
    spare.start();  // the next one warms up meanwhile
    p.pid = pid;
    p.state = "running";
    p.reason = "";
    p.started_at = now_s();
    p.launcher = "spare";
    return true;
  }

  void start(Proc& p) {
    if (start_zygote(p)) return;
    if (start_spare(p)) return;
    p.launcher = "exec";
    int pipefd[2];
    if (pipe2(pipefd, O_CLOEXEC) != 0) pipefd[0] = pipefd[1] = -1;
    pid_t pid = fork();
    if (pid == 0) {
      setsid();
      sigset_t none;
      sigemptyset(&none);
      sigprocmask(SIG_SETMASK, &none, nullptr);
      signal(SIGPIPE, SIG_DFL);
      if (!p.log.empty()) {
        int fd = open(p.log.c_str(), O_WRONLY | O_CREAT | O_APPEND, 0644);
        if (fd >= 0) {
          dup2(fd, 1);
          dup2(fd, 2);
          if (fd > 2) close(fd);
        }
      }
      int devnull = open("/dev/null", O_RDONLY);
      if (devnull >= 0) { dup2(devnull, 0); if (devnull > 2) close(devnull); }
      if (!p.cwd.empty() && chdir(p.cwd.c_str()) != 0) {
        fprintf(stderr, "pto-node-agent: chdir(%s): %s\n", p.cwd.c_str(), strerror(errno));
      }
      if (!p.cpus.empty()) {
        cpu_set_t set;
        CPU_ZERO(&set);
        for (int c : p.cpus) CPU_SET(c, &set);
        sched_setaffinity(0, sizeof set, &set);
      }
      std::vector<std::string> envs;
      for (auto& kv : p.env) envs.push_back(kv.first + "=" + kv.second);
      std::vector<char*> envp, argv;
      for (auto& e : envs) envp.push_back(const_cast<char*>(e.c_str()));
      envp.push_back(nullptr);
      for (auto& a : p.argv) argv.push_back(const_cast<char*>(a.c_str()));
      argv.push_back(nullptr);
      // PATH lookup with the container's PATH
      execvpe(argv[0], argv.data(), envp.data());
      int err = errno;
      fprintf(stderr, "pto-node-agent: exec %s: %s\n", argv[0], strerror(err));
      if (pipefd[1] >= 0) { ssize_t r = write(pipefd[1], &err, sizeof err); (void)r; }
      _exit(127);
    }
    if (pipefd[1] >= 0) close(pipefd[1]);
    int err = 0;
    if (pid > 0 && pipefd[0] >= 0) {
      // exec succeeded iff the CLOEXEC pipe closes without data
      ssize_t r = read(pipefd[0], &err, sizeof err);
      if (r <= 0) err = 0;
    }
    if (pipefd[0] >= 0) close(pipefd[0]);
    if (pid < 0) {
      p.state = "waiting";
      p.reason = "CreateContainerError";
      return;
    }
    p.pid = pid;
    p.state = "running";
    p.reason = err ? "StartError" : "";
    p.started_at = now_s();
  }

  Json spawn(const Json& req) {
    std::string id = req["id"].str();
    if (id.empty()) return err("spawn: missing id");
    auto it = procs.find(id);
    if (it != procs.end() && it->second.state != "terminated") return err("spawn: " + id + " already running");
    Proc p;
    p.id = id;
    for (auto& a : req["argv"].a) p.argv.push_back(a.str());
    if (p.argv.empty()) return err("spawn: empty argv");
    for (auto& kv : req["env"].o) p.env[kv.first] = kv.second.str();
    p.cwd = req["cwd"].str();
    p.log = req["log"].str();
    p.restart_policy = req["restart_policy"].str("Never");
    p.exec_only = req["launcher"].str("auto") == "exec";
    for (auto& c : req["cpus"].a) p.cpus.push_back((int)c.num());
    p.group = req["group"].str("");
    auto g = p.env.find("PTO_RESTART_GENERATION");
    p.gen_base = g == p.env.end() ? "0" : g->second;
    procs[id] = p;
    start(procs[id]);
    Json r = ok();
    r["pid"] = (long long)procs[id].pid;
    return r;
  }

  Json kill_(const Json& req) {
    auto it = procs.find(req["id"].str());
    if (it == procs.end()) return err("kill: unknown id");
    Proc& p = it->second;
    int sig = req.has("signal") ? (int)req["signal"].num() : SIGTERM;
    double grace = req.has("grace") ? req["grace"].num() : 10.0;
    bool restartable = req["restartable"].boolean(false);  // fault injection
    if (!restartable) p.stopping = true;
    if (p.state == "running" && p.pid > 0) {
      ::kill(-p.pid, sig);
      if (!restartable && sig != SIGKILL) p.kill_deadline = mono_s() + grace;
    } else if (p.state == "waiting" && !restartable) {
      p.state = "terminated";
      p.reason = "Killed";
      p.exit_code = 137;
      p.finished_at = now_s();
    }
    return ok();
  }

  Json remove(const Json& req) {
    auto it = procs.find(req["id"].str());
    if (it == procs.end()) return ok();
    if (it->second.state == "running") return err("remove: still running");
    procs.erase(it);
    return ok();
  }

  void on_exit(pid_t pid, int status) {
    if (pid == zygote.pid) {
      fprintf(stderr, "pto-node-agent: zygote %d exited (status %d); containers fall back to fork/exec\n",
              (int)pid, status);
      zygote.died();
      return;
    }
    if (pid == spare.pid) {  // died before it was used: exec'ed launches until a new one is warm
      fprintf(stderr, "pto-node-agent: spare interpreter %d exited (status %d)\n", (int)pid, status);
      spare.died();
      spare.start();
      return;
    }
    for (auto& kv : procs) {
      Proc& p = kv.second;
      if (p.pid != pid) continue;
      p.pid = -1;
      p.finished_at = now_s();
      if (WIFEXITED(status)) {
        p.exit_code = WEXITSTATUS(status);
        p.signal = 0;
      } else if (WIFSIGNALED(status)) {
        p.signal = WTERMSIG(status);
        p.exit_code = 128 + p.signal;
      }
      // the rest of the process group was killed by reap_one() before the
      // leader was reaped (its pid, hence the group id, was still reserved)
      bool restart = !p.stopping && (p.restart_policy == "Always" ||
                                     (p.restart_policy == "OnFailure" && p.exit_code != 0));
      const bool innocent = p.wave_killed;  // killed by its group's wave, did not fail itself
      p.wave_killed = false;
      if (restart) {
        p.last_exit_code = p.exit_code;
        p.last_finished_at = p.finished_at;
        // one restart per wave, charged to the member that failed: the
        // controller's backoffLimit sums restartCount over the job's pods
        // (pastBackoffLimit), so a wave must not count once per member
        double delay = innocent ? 0.0 : std::min(backoff_max, backoff_base * (double)(1 << std::min(p.restart_count, 16)));
        if (!innocent) p.restart_count += 1;
        p.state = "waiting";
        p.reason = "CrashLoopBackOff";
        p.restart_at = mono_s() + delay;
        if (!p.group.empty()) {
          Group& g = groups[p.group];
          if (!g.draining && p.exit_code != 0) begin_wave(p.group, p.id);
          if (g.draining) {  // restarts with the rest of its group
            p.held = true;
            p.held_delay = delay;
          }
        }
      } else {
        p.state = "terminated";
        p.reason = p.exit_code == 0 ? "Completed" : (p.stopping ? "Killed" : "Error");
      }
      return;
    }
  }

  // A member failed: every other running member of its group is killed
  // (it would otherwise sit in a collective with a dead peer, and the
  // restarted rank would rendezvous with a store that belongs to it).
  void begin_wave(const std::string& name, const std::string& culprit) {
    Group& g = groups[name];
    g.draining = true;
    g.wave += 1;
    g.drain_started = mono_s();
    int killed = 0;
    for (auto& kv : procs) {
      Proc& q = kv.second;
      if (q.group != name || q.id == culprit || q.stopping) continue;
      if (q.state == "running" && q.pid > 0) {
        q.wave_killed = true;
        ::kill(-q.pid, SIGKILL);
        ++killed;
      } else if (q.state == "waiting" && q.reason == "CrashLoopBackOff") {
        q.held = true;  // already owed a restart: it joins this wave
        q.held_delay = std::max(0.0, q.restart_at - mono_s());
      }
      // a member that already exited 0 is NOT revived: in Kubernetes a pod
      // whose containers all succeeded is terminal, and a succeeded Master
      // completes the job (reference status.go:99-106) -- reviving it would
      // rerun finished training over its outputs and move a Succeeded pod
      // back to Running.  The wave goes on without it.
    }
    fprintf(stderr, "pto-node-agent: group %s: %s failed, restart wave %d (%d member(s) stopped)\n",
            name.c_str(), culprit.c_str(), g.wave, killed);
  }

  // Restart a drained group: all held members at once, after the longest
  // back-off any of them is owed, under the wave's generation.
  void release_groups() {
    for (auto& gkv : groups) {
      Group& g = gkv.second;
      if (!g.draining) continue;
      bool live = false;
      double delay = 0;
      for (auto& kv : procs) {
        const Proc& q = kv.second;
        if (q.group != gkv.first) continue;
        if (q.state == "running") live = true;
        if (q.held) delay = std::max(delay, q.held_delay);
      }
      if (live) continue;
      const double at = mono_s() + delay;
      for (auto& kv : procs) {
        Proc& q = kv.second;
        if (q.group != gkv.first || !q.held) continue;
        q.held = false;
        q.restart_at = at;
        q.env["PTO_RESTART_GENERATION"] = q.gen_base + "." + std::to_string(g.wave);
      }
      g.draining = false;
    }
  }

  void tick() {
    release_groups();
    double t = mono_s();
    for (auto& kv : procs) {
      Proc& p = kv.second;
      if (p.state == "waiting" && p.reason == "CrashLoopBackOff" && !p.stopping && !p.held && t >= p.restart_at)
        start(p);
      if (p.state == "running" && p.kill_deadline > 0 && t >= p.kill_deadline && p.pid > 0) {
        ::kill(-p.pid, SIGKILL);
        p.kill_deadline = 0;
      }
    }
  }

  Json status(const Json& req) {
    Json out = ok();
    Json list = Json::array();
    std::string only = req["id"].str();
    for (auto& kv : procs) {
      if (!only.empty() && kv.first != only) continue;
      const Proc& p = kv.second;
      Json j = Json::object();
      j["id"] = p.id;
      j["pid"] = (long long)p.pid;
      j["state"] = p.state;
      j["reason"] = p.reason;
      j["exit_code"] = p.exit_code;
      j["signal"] = p.signal;
      j["restart_count"] = p.restart_count;
      j["started_at"] = p.started_at;
      j["finished_at"] = p.finished_at;
      j["last_exit_code"] = p.last_exit_code;
      j["last_finished_at"] = p.last_finished_at;
      j["launcher"] = p.launcher;
      j["group"] = p.group;
      j["held"] = p.held;
      auto g = p.env.find("PTO_RESTART_GENERATION");
      j["generation"] = g == p.env.end() ? std::string() : g->second;
      list.push(j);
    }
    out["procs"] = list;
    return out;
  }

  // ----------------------------------------------------------- GPUs ---
  Json gpus() {
    Json out = ok();
    Json list = Json::array();
    for (int g = 0; g < n_gpus; ++g) {
      Json j = Json::object();
      j["index"] = g;
      j["owner"] = gpu_owner[g];
      j["hbm_requested"] = gpu_hbm[g];
      j["hbm_total"] = hbm_per_gpu;
      j["numa_node"] = gpu_numa[g];
      list.push(j);
    }
    out["gpus"] = list;
    out["count"] = n_gpus;
    return out;
  }

  // all-or-nothing: {"requests":[{"owner":..,"count":k,"hbm":bytes}, ...]}
  Json alloc(const Json& req) {
    std::vector<std::string> owner = gpu_owner;
    std::vector<double> hbm = gpu_hbm;
    Json assigned = Json::object();
    for (auto& r : req["requests"].a) {
      std::string who = r["owner"].str();
      int k = (int)r["count"].num();
      double h = r["hbm"].num(0);
      if (h > hbm_per_gpu) return err("alloc: " + who + " requests more HBM than one GPU has");
      // already holding GPUs -> idempotent
      Json mine = Json::array();
      for (int g = 0; g < n_gpus; ++g)
        if (owner[g] == who) mine.push(g);
      if ((int)mine.a.size() >= k) { assigned[who] = mine; continue; }
      Json got = Json::array();
      for (int g = 0; g < n_gpus && (int)got.a.size() < k; ++g) {
        if (owner[g].empty()) {
          owner[g] = who;
          hbm[g] += h;
          got.push(g);
        }
      }
      if ((int)got.a.size() < k) {
        Json e = err("alloc: insufficient amd.com/gpu for gang (need " + std::to_string(k) + " for " + who + ")");
        e["unschedulable"] = true;
        return e;
      }
      assigned[who] = got;
    }
    gpu_owner = owner;
    gpu_hbm = hbm;
    Json out = ok();
    out["assigned"] = assigned;
    return out;
  }

  Json free_(const Json& req) {
    std::string who = req["owner"].str();
    int n = 0;
    for (int g = 0; g < n_gpus; ++g)
      if (gpu_owner[g] == who) { gpu_owner[g].clear(); gpu_hbm[g] = 0; ++n; }
    Json out = ok();
    out["freed"] = n;
    return out;
  }

  // TCP connect probe with timeout (init-container gate).
  Json probe(const Json& req) {
    std::string host = req["host"].str("127.0.0.1");
    std::string port = std::to_string((int)req["port"].num());
    double timeout = req.has("timeout") ? req["timeout"].num() : 0.5;
    addrinfo hints{}, *res = nullptr;
    hints.ai_socktype = SOCK_STREAM;
    Json out = ok();
    out["open"] = false;
    if (getaddrinfo(host.c_str(), port.c_str(), &hints, &res) != 0 || !res) return out;
    for (addrinfo* a = res; a; a = a->ai_next) {
      int fd = socket(a->ai_family, a->ai_socktype | SOCK_NONBLOCK, a->ai_protocol);
      if (fd < 0) continue;
      int rc = connect(fd, a->ai_addr, a->ai_addrlen);
      bool open_ = rc == 0;
      if (rc != 0 && errno == EINPROGRESS) {
        pollfd pf{fd, POLLOUT, 0};
        if (poll(&pf, 1, (int)(timeout * 1000)) == 1) {
          int e = 0;
          socklen_t l = sizeof e;
          getsockopt(fd, SOL_SOCKET, SO_ERROR, &e, &l);
          open_ = e == 0;
        }
      }
      close(fd);
      if (open_) { out["open"] = true; break; }
    }
    freeaddrinfo(res);
    return out;
  }

  static Json ok() { Json j = Json::object(); j["ok"] = true; return j; }
  static Json err(const std::string& m) {
    Json j = Json::object();
    j["ok"] = false;
    j["error"] = m;
    return j;
  }

  Json handle(const std::string& line) {
    Json req;
    try {
      req = Json::parse(line);
    } catch (std::exception& e) {
      return err(std::string("bad request: ") + e.what());
    }
    std::string op = req["op"].str();
    Json r;
    if (op == "ping") {
      r = ok();
      r["gpus"] = n_gpus;
      r["pid"] = (long long)getpid();
      Json z = Json::object();
      z["enabled"] = zygote.enabled();
      z["ready"] = zygote.ready;
      z["pid"] = (long long)zygote.pid;
      z["spawned"] = zygote.spawned;
      z["fallbacks"] = zygote.fallbacks;
      z["spare_ready"] = spare.ready;
      z["spares_used"] = spares_used;
      r["zygote"] = z;
    }
    else if (op == "spawn") r = spawn(req);
    else if (op == "kill") r = kill_(req);
    else if (op == "remove") r = remove(req);
    else if (op == "status") r = status(req);
    else if (op == "gpus") r = gpus();
    else if (op == "alloc") r = alloc(req);
    else if (op == "free") r = free_(req);
    else if (op == "probe") r = probe(req);
    else if (op == "shutdown") { quit = true; r = ok(); }
    else r = err("unknown op: " + op);
    if (req.has("seq")) r["seq"] = req["seq"];
    return r;
  }

  void kill_all() {
    for (auto& kv : procs)
      if (kv.second.state == "running" && kv.second.pid > 0) ::kill(-kv.second.pid, SIGKILL);
  }
};

struct Client {
  int fd;
  std::string inbuf;
};

static void usage() {
  fprintf(stderr,
          "usage: pto-node-agent (--socket PATH | --stdio) [--gpus N] [--hbm-per-gpu BYTES]\n"
          "                      [--backoff-base S] [--backoff-max S]\n"
          "                      [--zygote PYTHON [--zygote-pythonpath DIR]]\n");
}

// Reap one exited child, if any.  The child is first observed WITHOUT
// reaping it (WNOWAIT): while it is a zombie its pid -- and so its process
// group id (containers are session leaders) -- cannot be recycled, so
// SIGKILLing the group here can only hit the container's own leftovers,
// never an unrelated group that later took the same id.
static bool reap_one(Agent& ag) {
  siginfo_t si;
  memset(&si, 0, sizeof si);
  if (waitid(P_ALL, 0, &si, WEXITED | WNOHANG | WNOWAIT) != 0 || si.si_pid == 0) return false;
  const pid_t pid = si.si_pid;
  if (pid != ag.zygote.pid && pid != ag.spare.pid) ::kill(-pid, SIGKILL);
  int st = 0;
  if (waitpid(pid, &st, 0) != pid) return false;
  ag.on_exit(pid, st);
  return true;
}

int main(int argc, char** argv) {
  std::string sock_path;
  bool stdio = false;
  int forced_gpus = -1;
  Agent ag;
  for (int i = 1; i < argc; ++i) {
    std::string a = argv[i];
    auto next = [&]() -> std::string {
      if (i + 1 >= argc) { usage(); exit(2); }
      return argv[++i];
    };
    if (a == "--socket") sock_path = next();
    else if (a == "--stdio") stdio = true;
    else if (a == "--gpus") forced_gpus = atoi(next().c_str());
    else if (a == "--hbm-per-gpu") ag.hbm_per_gpu = atof(next().c_str());
    else if (a == "--backoff-base") ag.backoff_base = atof(next().c_str());
    else if (a == "--backoff-max") ag.backoff_max = atof(next().c_str());
    else if (a == "--zygote") ag.zygote.python = next();
    else if (a == "--zygote-pythonpath") ag.zygote.pypath = next();
    else if (a == "--version") { printf("pto-node-agent 0.1.0 (gfx950 / MI355X)\n"); return 0; }
    else { usage(); return 2; }
  }
  if (sock_path.empty() && !stdio) { usage(); return 2; }
  ag.discover_gpus(forced_gpus);

  sigset_t mask;
  sigemptyset(&mask);
  sigaddset(&mask, SIGCHLD);
  sigaddset(&mask, SIGTERM);
  sigaddset(&mask, SIGINT);
  sigprocmask(SIG_BLOCK, &mask, nullptr);
  int sfd = signalfd(-1, &mask, SFD_NONBLOCK | SFD_CLOEXEC);
  signal(SIGPIPE, SIG_IGN);
  // zygote-forked containers are orphaned by their forking parent: be their
  // reaper so waitpid() sees them like our own children
  prctl(PR_SET_CHILD_SUBREAPER, 1);
  ag.zygote.start();
  ag.spare.python = ag.zygote.python;
  ag.spare.pypath = ag.zygote.pypath;
  ag.spare.spare = true;
  ag.spare.start();

  int lfd = -1;
  std::vector<Client> clients;
  if (stdio) {
    int fl = fcntl(0, F_GETFL);
    fcntl(0, F_SETFL, fl | O_NONBLOCK);
    clients.push_back({0, ""});
  } else {
    lfd = socket(AF_UNIX, SOCK_STREAM | SOCK_CLOEXEC | SOCK_NONBLOCK, 0);
    sockaddr_un addr{};
    addr.sun_family = AF_UNIX;
    strncpy(addr.sun_path, sock_path.c_str(), sizeof(addr.sun_path) - 1);
    unlink(sock_path.c_str());
    if (bind(lfd, (sockaddr*)&addr, sizeof addr) != 0 || listen(lfd, 64) != 0) {
      perror("pto-node-agent: bind/listen");
      return 1;
    }
  }
  int signals_seen = 0;
  while (!ag.quit) {
    std::vector<pollfd> pfds;
    pfds.push_back({sfd, POLLIN, 0});
    if (lfd >= 0) pfds.push_back({lfd, POLLIN, 0});
    if (ag.zygote.fd >= 0 && !ag.zygote.ready) pfds.push_back({ag.zygote.fd, POLLIN, 0});
    if (ag.spare.fd >= 0 && !ag.spare.ready) pfds.push_back({ag.spare.fd, POLLIN, 0});
    for (auto& c : clients) pfds.push_back({c.fd, POLLIN, 0});
    poll(pfds.data(), pfds.size(), 50);
    ag.zygote.poll_ready();
    ag.spare.poll_ready();
    // signals
    signalfd_siginfo si;
    while (read(sfd, &si, sizeof si) == (ssize_t)sizeof si) {
      if (si.ssi_signo == SIGCHLD) {
        int st;
        pid_t pid;
        (void)st;
        (void)pid;
        while (reap_one(ag)) {
        }
      } else {
        // first SIGTERM/SIGINT: graceful stop; second: exit(1) (signals.go semantics)
        if (++signals_seen >= 2) { ag.kill_all(); return 1; }
        ag.quit = true;
      }
    }
    ag.tick();
    // accept
    if (lfd >= 0) {
      int cfd;
      while ((cfd = accept4(lfd, nullptr, nullptr, SOCK_NONBLOCK | SOCK_CLOEXEC)) >= 0) clients.push_back({cfd, ""});
    }
    // read requests
    for (size_t ci = 0; ci < clients.size();) {
      Client& c = clients[ci];
      char buf[65536];
      bool closed = false;
      while (true) {
        ssize_t r = read(c.fd, buf, sizeof buf);
        if (r > 0) { c.inbuf.append(buf, r); continue; }
        if (r == 0) closed = true;
        break;
      }
      size_t nl;
      while ((nl = c.inbuf.find('\n')) != std::string::npos) {
        std::string line = c.inbuf.substr(0, nl);
        c.inbuf.erase(0, nl + 1);
        if (line.empty()) continue;
        std::string reply = ag.handle(line).dump() + "\n";
        int ofd = (c.fd == 0) ? 1 : c.fd;
        size_t off = 0;
        while (off < reply.size()) {
          ssize_t w = write(ofd, reply.data() + off, reply.size() - off);
          if (w > 0) off += (size_t)w;
          else if (errno == EAGAIN) { pollfd pf{ofd, POLLOUT, 0}; poll(&pf, 1, 100); }
          else break;
        }
      }
      if (closed) {
        if (c.fd == 0) { ag.quit = true; break; }
        close(c.fd);
        clients.erase(clients.begin() + ci);
      } else {
        ++ci;
      }
    }
  }
  // graceful: terminate children, then reap (the zygote ends on EOF)
  if (ag.zygote.fd >= 0) {
    close(ag.zygote.fd);
    ag.zygote.fd = -1;
  }
  if (ag.spare.fd >= 0) {  // an unused spare ends on EOF too
    close(ag.spare.fd);
    ag.spare.fd = -1;
  }
  for (auto& kv : ag.procs)
    if (kv.second.state == "running" && kv.second.pid > 0) ::kill(-kv.second.pid, SIGTERM);
  double end = mono_s() + 5;
  while (mono_s() < end) {
    if (reap_one(ag)) continue;
    bool any = false;
    for (auto& kv : ag.procs) any |= kv.second.pid > 0;
    if (!any) break;
    usleep(20000);
  }
  ag.kill_all();
  if (!sock_path.empty()) unlink(sock_path.c_str());
  return 0;
}
