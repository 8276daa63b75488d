// wfsa: command-line driver with the reference's flags (src/main.cpp:66-108)
// for both optimizers (Hessian, the default, and QuasiNewton), running the
// objective/gradient (and the Hessian's count covariance) on the GPU.
//
//   wfsa -a A.wfsa -c C.corpus [-opt Hessian|QuasiNewton] [-e epochs] [-l eta]
//        [-tol t] [-i flags] [-n] [-eval] [-s] [-o out.wfsa] [-x] [-p] [-d device]
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <iostream>
#include <memory>
#include <string>
#include <vector>

#include "Corpus.hpp"
#include "Fsa.hpp"
#include "HessianLearner.hpp"
#include "Paths.hpp"
#include "QuasiNewtonLearner.hpp"

using namespace wfsa;

namespace {

void usage() {
    std::cerr << "usage: wfsa -a automaton.wfsa -c strings.corpus [options]\n"
                 "  -a, --automaton FILE   FSA to load\n"
                 "  -c, --corpus FILE      corpus to load\n"
                 "  -o, --output FILE      write the learned WFSA here (default stdout)\n"
                 "  -e, --epochs N         maximum optimization epochs (20)\n"
                 "  -l, --eta X            learning rate (1.0)\n"
                 "  -tol X                 halting tolerance (1e-6)\n"
                 "  -i, --init FLAGS       1 uniform, 2 normalize, 4 Lagrange init, 8 Hessian of the objective,\n"
                 "                         16 fill-reducing (minimum-degree) order of the sparse KKT factorisation, 32 exponential lambda\n"
                 "  -n, --normalize        normalize the automaton after optimization\n"
                 "  -eval                  evaluate the model after optimization\n"
                 "  -s, --suppress         do not print the learned FSA\n"
                 "  -x, --initx            read the initial x vector from stdin\n"
                 "  -opt NAME              Hessian (default) or QuasiNewton\n"
                 "  -p, --print            print the recognized paths, C, M, P and (Hessian) the KKT system to stderr\n"
                 "  -pr, --print-recognize print the recognized paths to stderr\n"
                 "  -r, --recognize N      path order of -p / -m >: 0 breadth-first (default), 1 depth-first\n"
                 "  -m, --matrix <FILE|>FILE  load the path matrices FILE.{C,M,P,prob,aux} instead of -a/-c,\n"
                 "                         or save them (after -a/-c: the paths enumerated on the host)\n"
                 "  -d, --device N         GPU to use (0)\n";
}

}  // namespace

int main(int argc, const char* argv[]) {
    std::string automaton, corpus_file, output, optimizer = "Hessian", matrices;
    int epochs = 20, initflags = 0, device = 0;
    double eta = 1.0, tol = 1e-6;
    bool normalize = false, suppress = false, evaluate = false, initx = false;
    bool print = false, print_recognize = false;
    int recognize = 0;   // 0: breadth-first, 1: depth-first (path order of -p / -m >)
    for (int i = 1; i < argc; ++i) {
        const std::string a = argv[i];
        auto next = [&]() -> const char* {
            if (i + 1 >= argc) {
                std::cerr << "missing value for " << a << std::endl;
                std::exit(1);
            }
            return argv[++i];
        };
        if (a == "-h" || a == "--help") { usage(); return 0; }
        else if (a == "-a" || a == "--automaton" || a == "--load") automaton = next();
        else if (a == "-c" || a == "--corpus") corpus_file = next();
        else if (a == "-o" || a == "--output") output = next();
        else if (a == "-e" || a == "--epoch" || a == "--epochs") epochs = std::atoi(next());
        else if (a == "-l" || a == "--learning" || a == "--eta") eta = std::atof(next());
        else if (a == "-tol" || a == "--tol" || a == "--tolerance") tol = std::atof(next());
        else if (a == "-i" || a == "--init") initflags = std::atoi(next());
        else if (a == "-opt" || a == "--optimizer") optimizer = next();
        else if (a == "-d" || a == "--device") device = std::atoi(next());
        else if (a == "-m" || a == "--matrix" || a == "--matrices") matrices = next();
        else if (a == "-n" || a == "--normalize") normalize = true;
        else if (a == "-eval" || a == "--eval" || a == "--evaluate") evaluate = true;
        else if (a == "-s" || a == "--suppress") suppress = true;
        else if (a == "-x" || a == "--initx" || a == "--initial") initx = true;
        else if (a == "-p" || a == "--print") print = true;
        else if (a == "-pr" || a == "--print-recognize") print_recognize = true;
        else if (a == "-r" || a == "--recognize") {
            recognize = std::atoi(next());
            if (recognize != 0 && recognize != 1) {
                std::cerr << "-r must be 0 (breadth-first) or 1 (depth-first)" << std::endl;
                return 1;
            }
        }
        else if (a == "-t" || a == "--thread" || a == "--threads") next();
        else { std::cerr << "unknown argument " << a << std::endl; usage(); return 1; }
    }
    if (optimizer != "QuasiNewton" && optimizer != "Hessian") {
        std::cerr << "optimizer must be Hessian or QuasiNewton, not \"" << optimizer << "\"" << std::endl;
        return 1;
    }
    try {
        std::unique_ptr<Learner> owner(optimizer == "Hessian" ? static_cast<Learner*>(new HessianLearner())
                                                               : static_cast<Learner*>(new QuasiNewtonLearner()));
        Learner& learner = *owner;
        learner.SetDevice(device);
        Fsa fsa;
        bool have_fsa = false;
        if (!matrices.empty() && matrices.front() == '<') {   // src/main.cpp:123-137: skip Corpus and Fsa
            std::cerr << "Loading matrices \"" << matrices.substr(1) << "\" ... ";
            if (!learner.LoadMatrices(matrices.substr(1)))
                throw LearnerError("Unable to load Learner from \"", matrices.substr(1), "\"");
            std::cerr << "done" << std::endl;
            std::cerr << "Info:\n\tparameters: " << learner.GetNumberOfParameters()
                      << "\n\tconstraints: " << learner.GetNumberOfConstraints()
                      << "\n\tstrings: " << learner.GetNumberOfStrings()
                      << "\n\tpaths: " << learner.GetNumberOfPaths()
                      << "\n\tcommon support: " << learner.GetCommonSupport()
                      << "\n\tunique paths: " << (learner.HasUniquePaths() ? "true" : "false") << std::endl;
        } else {
        Corpus corpus;
        if (FILE* f = std::fopen(corpus_file.c_str(), "rb")) {
            corpus.Read(f);
            std::fclose(f);
        } else {
            std::cerr << "\nUnable to open \"" << corpus_file << "\"!" << std::endl;
            return 1;
        }
        std::cerr << "Corpus:\n\tsize: " << corpus.size() << "\n\tsum: " << corpus.Sum();
        corpus.Renormalize();
        std::cerr << ", renormalized to " << corpus.Sum() << std::endl;
        if (FILE* f = std::fopen(automaton.c_str(), "rb")) {
            fsa.Read(f);
            std::fclose(f);
        } else {
            std::cerr << "\nUnable to open \"" << automaton << "\"!" << std::endl;
            return 1;
        }
        have_fsa = true;
        std::cerr << "Automaton:\n\tstates: " << fsa.GetNumberOfStates()
                  << "\n\ttransitions: " << fsa.GetNumberOfTransitions()
                  << "\n\temissions: " << fsa.GetNumberOfEmissions()
                  << "\n\tparameters: " << fsa.GetNumberOfParameters()
                  << "\n\tconstraints: " << fsa.GetNumberOfConstraints()
                  << "\n\tfree parameters: " << fsa.GetNumberOfFreeParameters() << std::endl;
        if (print || print_recognize) {   // src/main.cpp:178-203: every recognized path, on the host
            typedef std::pair<std::string, std::string> Path;   // (emitted string, state sequence)
            auto acc = [&](Path& h, const Fsa::NextState& t, const Fsa::NamedProb& e) {
                h.first += e.str;
                h.second += " -> ";
                h.second += t.next->first;
                if (e.str[0]) {
                    h.second += '"';
                    h.second += e.str;
                    h.second += '"';
                }
            };
            auto done = [](const Path& path) { std::fprintf(stderr, "%s: %s\n", path.first.c_str(), path.second.c_str()); };
            auto rec = make_recognizer<Path>(fsa, acc, done);
            for (const auto& word : corpus) rec.Recognize(word.first.c_str(), Path("", fsa.GetStartState()), recognize == 0);
        }
        learner.BuildFrom(fsa, corpus);
        if (print || (!matrices.empty() && matrices.front() == '>'))   // P / M for -p and for saving
            learner.EnumeratePaths(fsa, corpus, recognize == 0);
        std::cerr << "Recognize:\n\tstrings: " << learner.GetNumberOfStrings()
                  << "\n\tpaths: " << learner.GetNumberOfPaths()
                  << "\n\tcommon support: " << learner.GetCommonSupport()
                  << "\n\tunique paths: " << (learner.HasUniquePaths() ? "true" : "false")
                  << "\nAfter trimming:\n\tparameters: " << learner.GetNumberOfParameters()
                  << "\n\tconstraints: " << learner.GetNumberOfConstraints() << std::endl;
        }
        if (learner.GetNumberOfParameters() == 0) {
            std::cerr << "Empty automaton!" << std::endl;
            return 1;
        }
        if (learner.GetNumberOfStrings() == 0) {
            std::cerr << "Automaton cannot generate any of the strings!" << std::endl;
            return 1;
        }
        learner.Finalize();
        if (print) {   // src/main.cpp:231-239
            std::fputs("C:\n", stderr);
            learner.PrintC(stderr);
            std::fputs("M:\n", stderr);
            learner.PrintM(stderr);
            std::fputs("P:\n", stderr);
            learner.PrintP(stderr);
        }
        if (!matrices.empty() && matrices.front() == '>') {   // src/main.cpp:241-249
            std::cerr << "Saving matrices \"" << matrices.substr(1) << "\" ... ";
            std::cerr << (learner.SaveMatrices(matrices.substr(1)) ? "Done" : "Failed!") << std::endl;
        }
        std::cerr << "Initialize ... ";
        if (initx) {
            std::vector<double> x;
            while (std::cin && int32_t(x.size()) < learner.GetNumberOfParameters()) {
                x.emplace_back();
                std::cin >> x.back();
            }
            if (!std::cin) throw MyError("Cannot read initial x value!");
            learner.Init(initflags, x.data());
        } else {
            learner.Init(initflags);
        }
        std::cerr << "done" << std::endl;
        const int width = int(std::ceil(std::log10(epochs + 1)));
        if (epochs > 0) std::cerr << "Optimization:" << std::endl;
        for (int e = 1; e <= epochs; ++e) {
            if (e % 20 == 1) std::cerr << "epoch\t" << learner.GetOptimizationHeader() << std::endl;
            learner.OptimizationStep(eta, print);
            std::fprintf(stderr, "%0*d\t", width, e);
            const auto info = learner.GetOptimizationInfo();
            for (double x : info) {
                print_fixed_width(stderr, x, 9);
                std::fputs(" ", stderr);
            }
            std::cerr << std::endl;
            for (double x : info)
                if (!std::isfinite(x)) throw LearnerError(x, " detected at epoch ", e);
            if (learner.HaltCondition(tol)) break;
        }
        if (normalize) learner.Renormalize();
        if (evaluate) {
            const auto results = learner.GetOptimizationResult(print);
            std::cerr.precision(15);   // DBL_DIG
            std::cerr << "Result:";
            for (double x : results) std::cerr << ' ' << x;
            std::cerr << std::endl;
        }
        if (!suppress) {
            FILE* outf = output.empty() ? stdout : std::fopen(output.c_str(), "w");
            if (!outf) throw MyError("Unable to open output file \"", output, "\" for writing!");
            if (have_fsa) {
                learner.RewriteWeights(fsa);
                fsa.Dump(outf);
            } else {   // loaded from matrices (src/main.cpp:324-339): x, then lambda
                const int32_t n = learner.GetNumberOfParameters();
                const std::vector<double> lam = learner.GetLagrangeMultipliers();
                for (int32_t i = 0; i < n; ++i) std::fprintf(outf, i ? " %g" : "%g", learner.GetWeights()[i]);
                std::cout << std::endl;
                for (size_t c = 0; c < lam.size(); ++c) std::fprintf(outf, c ? " %g" : "%g", lam[c]);
                std::cout << std::endl;
            }
            if (outf != stdout) std::fclose(outf);
        }
    } catch (const std::exception& e) {
        std::fprintf(stderr, "%s\n", e.what());
        return 1;
    }
    return 0;
}
