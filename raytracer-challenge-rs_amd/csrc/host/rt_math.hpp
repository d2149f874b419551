// rt_math.hpp — C++ host mirror of the reference's math primitives:
// lib.rs (EPSILON, equal), vector.rs, point.rs, color.rs, ray.rs, matrix.rs,
// transform.rs. Same names, same operation order (left-associative Rust
// expressions, no FMA: host code is compiled with -ffp-contract=off), so the
// matrices handed to the device (inverses, camera) are bit-identical to the
// ones the Rust renderer computes.
#pragma once
#include <cmath>
#include <stdexcept>
#include <string>

namespace rt {

constexpr double EPSILON = 0.00001;  // lib.rs:18
inline bool equal(double a, double b) { return std::fabs(a - b) < EPSILON; }  // lib.rs:20-22

struct Vector;
struct Point {
  double x = 0, y = 0, z = 0;
  Point() = default;
  Point(double x_, double y_, double z_) : x(x_), y(y_), z(z_) {}
  static Point origin() { return Point(0, 0, 0); }
  bool operator==(const Point& o) const { return equal(x, o.x) && equal(y, o.y) && equal(z, o.z); }
};
struct Vector {
  double x = 0, y = 0, z = 0;
  Vector() = default;
  Vector(double x_, double y_, double z_) : x(x_), y(y_), z(z_) {}
  double magnitude() const { return std::sqrt(x * x + y * y + z * z); }  // vector.rs:21-23
  Vector normalize() const {                                             // vector.rs:25-28
    double m = magnitude();
    return Vector(x / m, y / m, z / m);
  }
  Vector reflect(const Vector& n) const;  // vector.rs:30-32
  bool operator==(const Vector& o) const { return equal(x, o.x) && equal(y, o.y) && equal(z, o.z); }
};
struct Color {
  double red = 0, green = 0, blue = 0;
  Color() = default;
  Color(double r, double g, double b) : red(r), green(g), blue(b) {}
  static Color black() { return Color(0, 0, 0); }
  static Color white() { return Color(1, 1, 1); }
  bool operator==(const Color& o) const {
    return equal(red, o.red) && equal(green, o.green) && equal(blue, o.blue);
  }
};

// point.rs:38-60
inline Point operator+(const Point& p, const Vector& v) { return Point(p.x + v.x, p.y + v.y, p.z + v.z); }
inline Vector operator-(const Point& a, const Point& b) { return Vector(a.x - b.x, a.y - b.y, a.z - b.z); }
inline Point operator-(const Point& p, const Vector& v) { return Point(p.x - v.x, p.y - v.y, p.z - v.z); }
// vector.rs:44-97
inline Vector operator+(const Vector& a, const Vector& b) { return Vector(a.x + b.x, a.y + b.y, a.z + b.z); }
inline Vector operator-(const Vector& a, const Vector& b) { return Vector(a.x - b.x, a.y - b.y, a.z - b.z); }
inline Vector operator-(const Vector& a) { return Vector(-a.x, -a.y, -a.z); }
inline Vector operator*(const Vector& a, double s) { return Vector(a.x * s, a.y * s, a.z * s); }
inline Vector operator/(const Vector& a, double s) { return Vector(a.x / s, a.y / s, a.z / s); }
inline double dot(const Vector& a, const Vector& b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
inline Vector cross(const Vector& a, const Vector& b) {  // vector.rs:103-109
  return Vector(a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x);
}
inline Vector Vector::reflect(const Vector& n) const { return *this - n * 2.0 * dot(*this, n); }
// color.rs:44-103
inline Color operator+(const Color& a, const Color& b) { return Color(a.red + b.red, a.green + b.green, a.blue + b.blue); }
inline Color operator-(const Color& a, const Color& b) { return Color(a.red - b.red, a.green - b.green, a.blue - b.blue); }
inline Color operator*(const Color& a, double s) { return Color(a.red * s, a.green * s, a.blue * s); }
inline Color operator*(const Color& a, const Color& b) { return Color(a.red * b.red, a.green * b.green, a.blue * b.blue); }

// ray.rs
struct Ray {
  Point origin;
  Vector direction;
  Ray() = default;
  Ray(const Point& o, const Vector& d) : origin(o), direction(d) {}
  Point position(double t) const { return origin + direction * t; }  // ray.rs:22-24
};

// matrix.rs: a general (<= 4x4) row-major matrix
class Matrix {
 public:
  Matrix() : rows_(4), cols_(4) { for (double& v : e_) v = 0.0; }
  Matrix(int rows, int cols) : rows_(rows), cols_(cols) {
    if (rows < 1 || rows > 4 || cols < 1 || cols > 4) throw std::invalid_argument("Matrix: 1..4 rows/cols");
    for (double& v : e_) v = 0.0;
  }
  static Matrix zero(int r, int c) { return Matrix(r, c); }
  static Matrix identity(int r, int c) {  // matrix.rs:28-36
    Matrix m(r, c);
    for (int i = 0; i < c && i < r; ++i) m(i, i) = 1.0;
    return m;
  }
  static Matrix from_slice(int r, int c, const double* v) {
    Matrix m(r, c);
    for (int i = 0; i < r * c; ++i) m.e_[i] = v[i];
    return m;
  }
  int rows() const { return rows_; }
  int columns() const { return cols_; }
  double& operator()(int i, int j) { return e_[i * cols_ + j]; }         // matrix.rs:75-77
  double operator()(int i, int j) const { return e_[i * cols_ + j]; }
  const double* data() const { return e_; }

  Matrix transpose() const {  // matrix.rs:79-89
    Matrix t(cols_, rows_);
    for (int i = 0; i < rows_; ++i)
      for (int j = 0; j < cols_; ++j) t(j, i) = (*this)(i, j);
    return t;
  }
  double determinant() const {  // matrix.rs:91-102
    if (rows_ == 2 && cols_ == 2) return (*this)(0, 0) * (*this)(1, 1) - (*this)(0, 1) * (*this)(1, 0);
    double det = 0.0;
    for (int c = 0; c < cols_; ++c) det += (*this)(0, c) * cofactor(0, c);
    return det;
  }
  Matrix submatrix(int row, int col) const {  // matrix.rs:104-120
    Matrix s(rows_ - 1, cols_ - 1);
    for (int i = 0; i < s.rows_; ++i)
      for (int j = 0; j < s.cols_; ++j) s(i, j) = (*this)(i < row ? i : i + 1, j < col ? j : j + 1);
    return s;
  }
  double minor(int r, int c) const { return submatrix(r, c).determinant(); }  // :122-124
  double cofactor(int r, int c) const { return (r + c) % 2 == 1 ? -minor(r, c) : minor(r, c); }  // :126-132
  bool is_invertible() const { return !equal(determinant(), 0.0); }  // :134-136
  Matrix inverse() const {  // matrix.rs:138-153
    if (!is_invertible() || rows_ != cols_) throw std::domain_error("Matrix::inverse: not invertible");
    Matrix inv(rows_, cols_);
    double det = determinant();
    for (int i = 0; i < rows_; ++i)
      for (int j = 0; j < cols_; ++j) inv(j, i) = cofactor(i, j) / det;
    return inv;
  }
  bool operator==(const Matrix& o) const {  // matrix.rs:201-208 (zip semantics)
    int n = rows_ * cols_, m = o.rows_ * o.cols_;
    for (int i = 0; i < n && i < m; ++i)
      if (!equal(e_[i], o.e_[i])) return false;
    return true;
  }
  bool operator!=(const Matrix& o) const { return !(*this == o); }
  // fluent API (matrix.rs:155-187): each prepends, `t * self`
  Matrix translate(double x, double y, double z) const;
  Matrix scale(double x, double y, double z) const;
  Matrix rotate_x(double r) const;
  Matrix rotate_y(double r) const;
  Matrix rotate_z(double r) const;
  Matrix shear(double xy, double xz, double yx, double yz, double zx, double zy) const;

 private:
  int rows_, cols_;
  double e_[16];
};

inline Matrix operator*(const Matrix& a, const Matrix& b) {  // matrix.rs:210-230
  if (a.columns() != b.rows()) throw std::invalid_argument("Matrix multiply: shape mismatch");
  Matrix m(a.rows(), b.columns());
  for (int row = 0; row < a.rows(); ++row)
    for (int col = 0; col < b.columns(); ++col) {
      double c = 0.0;
      for (int i = 0; i < a.columns(); ++i) c += a(row, i) * b(i, col);
      m(row, col) = c;
    }
  return m;
}
inline Point operator*(const Matrix& m, const Point& p) {  // matrix.rs:232-245
  return Point(m(0, 0) * p.x + m(0, 1) * p.y + m(0, 2) * p.z + m(0, 3),
               m(1, 0) * p.x + m(1, 1) * p.y + m(1, 2) * p.z + m(1, 3),
               m(2, 0) * p.x + m(2, 1) * p.y + m(2, 2) * p.z + m(2, 3));
}
inline Vector operator*(const Matrix& m, const Vector& v) {  // matrix.rs:247-260
  return Vector(m(0, 0) * v.x + m(0, 1) * v.y + m(0, 2) * v.z,
                m(1, 0) * v.x + m(1, 1) * v.y + m(1, 2) * v.z,
                m(2, 0) * v.x + m(2, 1) * v.y + m(2, 2) * v.z);
}
inline Ray transform(const Ray& r, const Matrix& m) { return Ray(m * r.origin, m * r.direction); }  // ray.rs:26-28

// transform.rs
inline Matrix translation(double x, double y, double z) {  // :7-15
  Matrix t = Matrix::identity(4, 4);
  t(0, 3) = x; t(1, 3) = y; t(2, 3) = z;
  return t;
}
inline Matrix scaling(double x, double y, double z) {  // :17-25
  Matrix s = Matrix::identity(4, 4);
  s(0, 0) = x; s(1, 1) = y; s(2, 2) = z;
  return s;
}
inline Matrix rotation_x(double r) {  // :27-36
  Matrix m = Matrix::identity(4, 4);
  m(1, 1) = std::cos(r); m(1, 2) = -std::sin(r); m(2, 1) = std::sin(r); m(2, 2) = std::cos(r);
  return m;
}
inline Matrix rotation_y(double r) {  // :38-47
  Matrix m = Matrix::identity(4, 4);
  m(0, 0) = std::cos(r); m(0, 2) = std::sin(r); m(2, 0) = -std::sin(r); m(2, 2) = std::cos(r);
  return m;
}
inline Matrix rotation_z(double r) {  // :49-58
  Matrix m = Matrix::identity(4, 4);
  m(0, 0) = std::cos(r); m(0, 1) = -std::sin(r); m(1, 0) = std::sin(r); m(1, 1) = std::cos(r);
  return m;
}
inline Matrix shearing(double xy, double xz, double yx, double yz, double zx, double zy) {  // :60-71
  Matrix s = Matrix::identity(4, 4);
  s(0, 1) = xy; s(0, 2) = xz; s(1, 0) = yx; s(1, 2) = yz; s(2, 0) = zx; s(2, 1) = zy;
  return s;
}
inline Matrix view_transform(const Point& from, const Point& to, const Vector& up) {  // :73-90
  Vector forward = (to - from).normalize();
  Vector upn = up.normalize();
  Vector left = cross(forward, upn);
  Vector true_up = cross(left, forward);
  const double o[16] = {left.x, left.y, left.z, 0.0,
                        true_up.x, true_up.y, true_up.z, 0.0,
                        -forward.x, -forward.y, -forward.z, 0.0,
                        0.0, 0.0, 0.0, 1.0};
  return Matrix::from_slice(4, 4, o) * translation(-from.x, -from.y, -from.z);
}
inline Matrix Matrix::translate(double x, double y, double z) const { return rt::translation(x, y, z) * *this; }
inline Matrix Matrix::scale(double x, double y, double z) const { return rt::scaling(x, y, z) * *this; }
inline Matrix Matrix::rotate_x(double r) const { return rt::rotation_x(r) * *this; }
inline Matrix Matrix::rotate_y(double r) const { return rt::rotation_y(r) * *this; }
inline Matrix Matrix::rotate_z(double r) const { return rt::rotation_z(r) * *this; }
inline Matrix Matrix::shear(double xy, double xz, double yx, double yz, double zx, double zy) const {
  return rt::shearing(xy, xz, yx, yz, zx, zy) * *this;
}

}  // namespace rt
