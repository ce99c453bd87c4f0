// leja.hpp -- Newton-basis set-up (modified Leja ordering, change-of-basis).
#pragma once

#include <complex>
#include <string>
#include <vector>

namespace cal {
namespace leja {

int count_multiplicities(const std::vector<std::complex<double>>& x, int n, bool cplx,
                         std::vector<std::complex<double>>& y, std::vector<double>& mults);
int modified_leja(std::vector<std::complex<double>> x, int n, const std::vector<double>& mults,
                  std::vector<std::complex<double>>& y, std::vector<int>& outidx, std::string& err);
int real_leja(const std::vector<std::complex<double>>& x, std::vector<std::complex<double>>& y,
              std::vector<int>& outidx, std::string& err);
// B is (s+1) x s column-major.
int newton_basis_matrix(int s, const std::vector<std::complex<double>>& lam, int modifiedp, std::vector<double>& B,
                        std::string& err);

}  // namespace leja
}  // namespace cal
